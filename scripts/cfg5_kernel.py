#!/usr/bin/env python3
"""cfg5 kernel alone (for PMC passes): 32 768 chains of gmm2, an 8-step
warm-up launch, then one 2000-step launch with the trace."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
from oracle.workloads import golden_init  # noqa: E402
from probayes_amd import Engine  # noqa: E402

eng = Engine(oracle.golden_spec('gmm2'))
eng.init_chains(golden_init('gmm2', 32768))
eng.set_rng('philox', seed=11)
eng.set_collect(moments=False)
eng.run(8)
eng.alloc_trace(2000, 1)
eng.run(2000)
print('kernel ms', eng.last_run_ms())
eng.close()
