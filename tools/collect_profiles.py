"""Copy one scripts/gpu_check.sh run (gpurun_out/) into profiles/<tag>_*.

usage: python tools/collect_profiles.py <tag>     e.g. r01h

Writes the rocprofv3 kernel stats / traces, the PMC counter passes, the bench
lines and two traffic summaries: the cfg2 headline kernel and the cfg3
production Gibbs kernel.  FETCH_SIZE is doubled per MI355X_MICROARCH.md (gfx950
counts half of a wide coalesced read); WRITE_SIZE is taken as reported (KiB).
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, 'gpurun_out')
PROF = os.path.join(OUT, 'prof')


def counters(path, sub):
  rows = [r for r in csv.DictReader(open(path)) if sub in r['Kernel_Name']]
  return [float(r['Counter_Value']) for r in rows], rows


def main(tag):
  dst = lambda name: os.path.join(ROOT, 'profiles', '{}_{}'.format(tag, name))
  copies = {'trace/run_kernel_stats.csv': 'kernel_stats.csv',
            'trace/run_kernel_trace.csv': 'kernel_trace.csv',
            'wl/run_kernel_stats.csv': 'workloads_kernel_stats.csv',
            'fetch/run_counter_collection.csv': 'pmc_fetch_size.csv',
            'write/run_counter_collection.csv': 'pmc_write_size.csv',
            'sq1/run_counter_collection.csv': 'pmc_sq1.csv',
            'sq2/run_counter_collection.csv': 'pmc_sq2.csv',
            'sq3/run_counter_collection.csv': 'pmc_sq3.csv',
            'wl_fetch/run_counter_collection.csv': 'cfg3_pmc_fetch_size.csv',
            'wl_write/run_counter_collection.csv': 'cfg3_pmc_write_size.csv',
            'lik_fetch/run_counter_collection.csv': 'lik_pmc_fetch_size.csv',
            'lik_write/run_counter_collection.csv': 'lik_pmc_write_size.csv'}
  for src, name in copies.items():
    if os.path.exists(os.path.join(PROF, src)):
      shutil.copy(os.path.join(PROF, src), dst(name))
  with open(dst('bench_lines.jsonl'), 'w') as f:
    for log in ('bench.log', 'bench_xo.log', 'workloads.log'):
      for line in open(os.path.join(OUT, log)):
        if line.startswith('{'):
          f.write(line)

  # cfg2 headline: mh_pair_kernel<10, PHILOX>, 65 536 chains x 250 steps/launch
  k = 'mh_pair_kernel<10, 1>'
  fetch, _ = counters(os.path.join(PROF, 'fetch/run_counter_collection.csv'), k)
  write, _ = counters(os.path.join(PROF, 'write/run_counter_collection.csv'), k)
  stats = {r['Name']: r for r in csv.DictReader(
      open(os.path.join(PROF, 'trace/run_kernel_stats.csv')))}
  st = [v for n, v in stats.items() if k in n][0]
  fk, wk = sum(fetch) / len(fetch), sum(write) / len(write)
  b = (2 * fk + wk) * 1024
  alg = 88.125 * 65536 * 250
  json.dump({'kernel': 'mh_pair_kernel<10, PHILOX>', 'chains': 65536,
             'steps_per_launch': 250, 'fetch_size_kb': fk, 'write_size_kb': wk,
             'bytes_per_launch': b, 'algorithmic_bytes_per_launch': alg,
             'traffic_over_algorithmic': b / alg,
             'avg_launch_ns': float(st['AverageNs']), 'dispatches': len(fetch),
             'source': 'scripts/gpu_check.sh: rocprofv3 --pmc FETCH_SIZE / --pmc '
                       'WRITE_SIZE in separate passes; FETCH_SIZE doubled (gfx950 '
                       'counts half of a wide coalesced read, MI355X_MICROARCH.md)'},
            open(dst('traffic.json'), 'w'), indent=1)

  # cfg3 production Gibbs: the 2048-step launch (largest WRITE_SIZE dispatch)
  k = 'gibbs_fast_kernel<8, 2>'
  fetch, _ = counters(os.path.join(PROF, 'wl_fetch/run_counter_collection.csv'), k)
  write, _ = counters(os.path.join(PROF, 'wl_write/run_counter_collection.csv'), k)
  i = max(range(len(write)), key=lambda j: write[j])
  b = (2 * fetch[i] + write[i]) * 1024
  alg = 32768 * 2048 * 72.125  # x[8] + v.prob fp64 + 1 accept bit per coordinate-step
  wl = {r['Name']: r for r in csv.DictReader(
      open(os.path.join(PROF, 'wl/run_kernel_stats.csv')))}
  st = [v for n, v in wl.items() if k in n]
  json.dump({'kernel': k, 'chains': 32768, 'steps_per_launch': 2048,
             'fetch_size_kb': fetch[i], 'write_size_kb': write[i],
             'bytes_per_launch': b, 'algorithmic_bytes_per_launch': alg,
             'traffic_over_algorithmic': b / alg,
             'launch_ns': float(st[0]['MaxNs']) if st else None,
             'source': 'scripts/gpu_check.sh prof_wl_fetch / prof_wl_write '
                       '(bench_workloads.py --only cfg3); launch_ns = the '
                       '2048-step dispatch (MaxNs of prof_wl)'},
            open(dst('cfg3_gibbs_traffic.json'), 'w'), indent=1)


if __name__ == '__main__':
  main(sys.argv[1])
