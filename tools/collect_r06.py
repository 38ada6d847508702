"""Copy scripts/profile_r06.sh's output (gpurun_out/prof6) into profiles/:
per shape the kernel stats / trace CSVs, the FETCH_SIZE / WRITE_SIZE / SQ
passes, the bench lines, and a traffic JSON keyed by (kernel instance, srv,
chains, steps per launch or command, rng) that bench.py's measured_traffic
reads.  FETCH_SIZE is doubled per MI355X_MICROARCH.md (gfx950 counts half of
a wide coalesced read); WRITE_SIZE is taken as reported (KiB).

usage: python tools/collect_r06.py <tag>      e.g. r06a

Shapes:
  * s20srv -- the driver's shape as bench.py runs it: the timed 20 steps are
    a command to the resident server, whose kernel
    (mh_pair_kernel<10, 1, false, true, true, true>: FULL, SRV) is ONE
    dispatch for the server's life -- the warm-up's one-step commands and the
    timed 20-step command, plus the polls between them.  Its FETCH / WRITE
    bytes are divided over the steps commanded in that life (read from the
    pass's own bench line: commands - 1 one-step warm-ups + the timed steps)
    and scaled to one 20-step command;
  * s20 -- the same 20 steps launched (PBH_SERVER=0): the last FULL dispatch;
  * s1000 -- the default shape, 250-step launches: the 4 timed dispatches.
Every traffic JSON carries the sha256 of the library the passes ran
(gpurun_out/prof6/lib.sha256): bench.py takes roofline.traffic only from a
profile of the binary it loads, and of the instance it timed.
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, 'gpurun_out', 'prof6')
LAUNCHED = 'mh_pair_kernel<10, 1, false, true, true, false>'   # FULL, loc 0, launched
SERVER = 'mh_pair_kernel<10, 1, false, true, true, true>'      # FULL, loc 0, SRV
ALG = 88.125 * 65536   # algorithmic bytes per cfg2 step of 65 536 chains


def rows(path, kernel):
  return [r for r in csv.DictReader(open(path)) if kernel in r['Kernel_Name']]


def sq_summary(path, kernel, last):
  by = {}
  for r in rows(path, kernel):
    by.setdefault(r['Counter_Name'], []).append(float(r['Counter_Value']))
  return {k: sum(v[-last:]) / last for k, v in by.items()}


def bench_lines(*logs):
  out = []
  for log in logs:
    if os.path.exists(log):
      out += [json.loads(l) for l in open(log) if l.startswith('{')]
  return out


def copy_shape(tag, shape):
  src = os.path.join(PROF, shape)
  dst = lambda name: os.path.join(ROOT, 'profiles', '{}_{}_{}'.format(tag, shape, name))
  for a, b in (('trace/run_kernel_stats.csv', 'kernel_stats.csv'),
               ('trace/run_kernel_trace.csv', 'kernel_trace.csv'),
               ('fetch/run_counter_collection.csv', 'pmc_fetch_size.csv'),
               ('write/run_counter_collection.csv', 'pmc_write_size.csv'),
               ('sq/run_counter_collection.csv', 'pmc_sq.csv')):
    if os.path.exists(os.path.join(src, a)):
      shutil.copy(os.path.join(src, a), dst(b))
  logs = [os.path.join(src, f) for f in sorted(os.listdir(src)) if f.endswith('.log')]
  with open(dst('bench_lines.jsonl'), 'w') as f:
    for line in bench_lines(*logs):
      f.write(json.dumps(line) + '\n')
  return src


def main(tag):
  sha = open(os.path.join(PROF, 'lib.sha256')).read().split()[0]
  src = os.path.join(PROF, 'steps.txt')
  if os.path.exists(src):
    shutil.copy(src, os.path.join(ROOT, 'profiles', '{}_steps.txt'.format(tag)))
  for shape, spl in (('s20', 20), ('s1000', 250)):
    src = copy_shape(tag, shape)
    tr = rows(os.path.join(src, 'trace/run_kernel_trace.csv'), LAUNCHED)
    dur = [int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in tr]
    fetch = [float(r['Counter_Value']) for r in
             rows(os.path.join(src, 'fetch/run_counter_collection.csv'), LAUNCHED)]
    write = [float(r['Counter_Value']) for r in
             rows(os.path.join(src, 'write/run_counter_collection.csv'), LAUNCHED)]
    k = 1 if shape == 's20' else 4   # the timed FULL dispatches
    fk, wk = sum(fetch[-k:]) / k, sum(write[-k:]) / k
    b = (2 * fk + wk) * 1024
    alg = ALG * spl
    json.dump({'kernel': 'mh_pair_kernel<10, PHILOX, MOM=0, FULL>', 'srv': False,
               'chains': 65536, 'steps_per_launch': spl, 'rng': 'philox',
               'fetch_size_kb': fk, 'write_size_kb': wk,
               'bytes_per_launch': b, 'algorithmic_bytes_per_launch': alg,
               'traffic_over_algorithmic': b / alg,
               'avg_launch_ns_trace': sum(dur[-k:]) / k, 'dispatches': k,
               'lib_sha256': sha,
               'sq_per_dispatch': sq_summary(os.path.join(src, 'sq/run_counter_collection.csv'),
                                             LAUNCHED, k),
               'source': 'scripts/profile_r06.sh ({}, PBH_SERVER=0): rocprofv3 --pmc '
                         'FETCH_SIZE / --pmc WRITE_SIZE in separate passes of bench.py; '
                         'FETCH_SIZE doubled (MI355X_MICROARCH.md)'.format(shape)},
              open(os.path.join(ROOT, 'profiles', '{}_traffic_{}.json'.format(tag, shape)),
                   'w'), indent=1)
  # the server's one dispatch (s20srv)
  src = copy_shape(tag, 's20srv')
  if os.path.exists(os.path.join(src, 'probe.jsonl')):
    shutil.copy(os.path.join(src, 'probe.jsonl'),
                os.path.join(ROOT, 'profiles', '{}_s20srv_server_probe.jsonl'.format(tag)))
  passes = {}
  for name in ('fetch', 'write', 'sq'):
    line = bench_lines(os.path.join(src, 'bench_{}.log'.format(name)))[0]
    cmds = line['server']['commands']
    assert line['server']['launches'] == 1, line['server']
    life = (cmds - 1) + line['steps']   # one-step warm-up commands + the timed one
    r = rows(os.path.join(src, name, 'run_counter_collection.csv'), SERVER)
    passes[name] = (r, life, line)
  (fr, flife, fline), (wr, wlife, _), (sr, slife, _) = passes['fetch'], passes['write'], passes['sq']
  assert len([r for r in fr]) == 1 and len(wr) == 1, (len(fr), len(wr))
  fk, wk = float(fr[0]['Counter_Value']), float(wr[0]['Counter_Value'])
  life_bytes = 2 * fk * 1024 * 20 / flife + wk * 1024 * 20 / wlife   # per 20-step command
  sq = {}
  for r in sr:
    sq[r['Counter_Name']] = float(r['Counter_Value'])
  json.dump({'kernel': 'mh_pair_kernel<10, PHILOX, MOM=0, FULL, SRV>', 'srv': True,
             'chains': 65536, 'steps_per_launch': 20, 'rng': 'philox',
             'life_steps_fetch_pass': flife, 'life_steps_write_pass': wlife,
             'life_steps_sq_pass': slife,
             'fetch_size_kb_life': fk, 'write_size_kb_life': wk,
             'dispatch_ns_fetch_pass': int(fr[0]['End_Timestamp']) - int(fr[0]['Start_Timestamp']),
             'bytes_per_launch': life_bytes,
             'algorithmic_bytes_per_launch': ALG * 20,
             'traffic_over_algorithmic': life_bytes / (ALG * 20),
             'lib_sha256': sha,
             'sq_life': sq,
             'events_us_fetch_pass': fline.get('events_us'),
             'source': 'scripts/profile_r06.sh (s20srv, the bench as the driver runs it): '
                       'rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE over the server '
                       'kernel\'s one dispatch (its whole life: the one-step warm-up '
                       'commands, the timed 20-step command, the polls between them, the '
                       'state load and store); bytes x 20 / steps commanded in the life; '
                       'FETCH_SIZE doubled (MI355X_MICROARCH.md)'},
            open(os.path.join(ROOT, 'profiles', '{}_traffic_s20srv.json'.format(tag)), 'w'),
            indent=1)
  for name in ('bench_driver', 'bench_default'):
    with open(os.path.join(ROOT, 'profiles', '{}_{}.jsonl'.format(tag, name)), 'w') as f:
      for line in bench_lines(os.path.join(PROF, name + '.log')):
        f.write(json.dumps(line) + '\n')


if __name__ == '__main__':
  main(sys.argv[1])
