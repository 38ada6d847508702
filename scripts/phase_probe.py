#!/usr/bin/env python3
"""Where the fixed part of a short cfg2 launch goes, from inside the FULL
pair kernel: the probe build (libpbhip_ph.so, -DPBH_PHASES) stamps every
wave's real-time clock (100 MHz) at entry, after the LDS tables + state
loads, after the first pair's draws, after the step loop and after the final
state stores.  Per launch length, prints the spread of each phase over the
2 048 waves relative to the first wave's entry, next to the HIP-event time.
usage: PBHIP_LIB=probayes_amd/libpbhip_ph.so phase_probe.py TAG"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from probayes_amd import Engine, _lib  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else ''
if os.environ.get('PHASE_WORKLOAD', 'cfg2') == 'gmm2':
  # cfg5's share: the quad GMM kernel, 4 lanes per chain (scripts/bench_workloads.py)
  import oracle  # noqa: E402  (the model description only)
  N = int(os.environ.get('PHASE_N', 32768))
  waves = N // 16
  eng = Engine(oracle.golden_spec('gmm2'))
  eng.init_chains(oracle.workloads.golden_init('gmm2', N))
  lens = [4, 20, 100, 2000]
else:
  N = int(os.environ.get('PHASE_N', 65536))
  waves = N // 32
  eng = Engine(bench.cfg2_spec())
  eng.init_chains(np.zeros((N, bench.D)))
  lens = [1, 2, 4, 8, 20, 40, 100, 250]
eng.set_rng('philox', seed=7)
eng.set_collect(moments=False)
eng.alloc_trace(6 + 4 * sum(lens) + 64, 1)
lib = _lib.load()
raw = {}
dump = lib.pbh_phase_dump
dump.restype = ctypes.c_int
dump.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int64]
buf = np.zeros(waves * 8, np.uint64)
for _ in range(4):
  eng.run(1)
eng.sync()
for m in lens:
  for rep in range(3):
    if eng.trace_len() % 4:   # keep launches group-aligned (FULL's common case)
      eng.run(4 - eng.trace_len() % 4)
      eng.sync()
    eng.run(m, steps_per_launch=max(lens))
    eng.sync()
    ms, _ = eng.last_run_ms()
    rc = dump(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), buf.size)
    if rc:
      raise SystemExit('pbh_phase_dump -> {}'.format(rc))
    w8 = buf.reshape(waves, 8).astype(np.int64)
    st = w8[:, [0, 1, 2, 5, 6, 7, 3]].copy()   # entry, loaded, drawn, q1..q3, end
    # 'drawn' / quarter stamps exist only where the loop over whole pairs runs
    for k in (2, 3, 4, 5):
      st[:, k] = np.where(st[:, k] == 0, st[:, k - 1], st[:, k])
    if (st[:, [0, 1, 6]] == 0).any():
      raise SystemExit('missing stamps: {} waves'.format(int((st == 0).any(1).sum())))
    t0 = st[:, 0].min()
    us = (st - t0) * 0.01   # 100 MHz ticks -> us
    # the wave's slot on its SIMD: HW_ID.WAVE_ID [3:0]; the SIMD itself is
    # HW_ID [15:4] (simd, pipe, cu, sh, se) + XCC_ID (word 4 bits 32..35)
    w4 = buf.reshape(waves, 8)[:, 4].astype(np.uint64)
    hw = (((w4 >> np.uint64(4)) & np.uint64(0xFFF)) |
          (((w4 >> np.uint64(32)) & np.uint64(0xF)) << np.uint64(12))).astype(np.int64)
    slot = (w4 & np.uint64(0xF)).astype(np.int64)
    order = np.lexsort((slot, hw))
    same = np.concatenate([[False], hw[order][1:] == hw[order][:-1]])
    # the waves of one SIMD in one workgroup? (wave index // waves per WG)
    wpg = int(os.environ.get('PHASE_WPG', '4'))
    grp = np.arange(len(hw)) // wpg
    pair_same_wg = float(np.mean(grp[order][1:][same[1:]] == grp[order][:-1][same[1:]])) \
        if same.any() else float('nan')
    row = {'tag': tag, 'steps': m, 'rep': rep, 'events_us': ms * 1e3,
           'simd_pairs_same_wg': pair_same_wg}
    for k, name in enumerate(['entry', 'loaded', 'drawn', 'q1', 'q2', 'q3', 'loop_end']):
      row[name] = [round(float(np.percentile(us[:, k], q)), 2) for q in (0, 50, 100)]
      row[name + '_slots'] = [round(float(np.median(us[slot == v, k])), 2) for v in (0, 1)]
    print(json.dumps(row), flush=True)
    raw['s{}_r{}'.format(m, rep)] = buf.reshape(waves, 8).copy()
eng.close()
out = os.environ.get('PHASE_RAW')
if out:
  np.savez_compressed(out, **raw)
