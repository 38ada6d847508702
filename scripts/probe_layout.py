#!/usr/bin/env python3
"""Does the trace row stride matter?  cfg2 at 250 steps/launch, trace on and
off, for chain counts whose fp64 row stride is / is not a multiple of a
large power of two."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'scripts'))
from launch_probe import probe  # noqa: E402

if __name__ == '__main__':
  for chains in (65536, 65536 + 64, 65536 + 512, 65536 - 64):
    for trace in (True, False):
      probe('philox', False, 250, 6, None, trace=trace, chains=chains)
  probe('philox', False, 20, 20, None, trace=True, chains=65536)
  probe('philox', False, 20, 20, None, trace=True, chains=65536 + 64)
