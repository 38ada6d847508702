#!/usr/bin/env python3
"""Where the device ESS call's wall time goes (cfg5 trace: 32 768 chains x 2
dims, records [500, 2000)): the whole Engine.trace_ess call, the C call with
no copy-out (kernels + launch + sync), and the C call with the copy-out;
ten calls each, min and median in ms."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
from oracle.workloads import golden_init  # noqa: E402
from probayes_amd import Engine, _lib  # noqa: E402

eng = Engine(oracle.golden_spec('gmm2'))
eng.init_chains(golden_init('gmm2', 32768))
eng.set_rng('philox', seed=11)
eng.set_collect(moments=False)
eng.alloc_trace(2000, 1)
eng.run(2000, steps_per_launch=250)
eng.sync()
eng.trace_ess(500)
out = np.empty((2, 32768))


def timeit(fn, reps=10):
  ts = []
  for _ in range(reps):
    t0 = time.perf_counter()
    fn()
    ts.append((time.perf_counter() - t0) * 1e3)
  return round(min(ts), 4), round(float(np.median(ts)), 4)


lib = _lib.load()
res = {
    'engine_call': timeit(lambda: eng.trace_ess(500)),
    'c_no_copy': timeit(lambda: _lib.call('pbh_trace_ess', eng._h, ctypes.c_int64(500),
                                          ctypes.c_int64(1500), None)),
    'c_copy_reused_out': timeit(lambda: _lib.call(
        'pbh_trace_ess', eng._h, ctypes.c_int64(500), ctypes.c_int64(1500),
        out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))),
    'empty_sync': timeit(lambda: eng.sync()),
}
print(res)
eng.close()
