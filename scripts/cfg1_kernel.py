#!/usr/bin/env python3
"""cfg1 kernel alone (for PMC passes): 32 768 chains of metrohast_norm1d, an 8-step
warm-up launch, then one 1000-step launch with the trace."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
from oracle.workloads import golden_init  # noqa: E402
from probayes_amd import Engine  # noqa: E402

eng = Engine(oracle.golden_spec('metrohast_norm1d'))
eng.init_chains(golden_init('metrohast_norm1d', 65536))
eng.set_rng('philox', seed=11)
eng.set_collect(moments=False)
eng.run(8)
eng.alloc_trace(1000, 1)
eng.run(1000)
print('kernel ms', eng.last_run_ms())
eng.close()
