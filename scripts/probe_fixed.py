#!/usr/bin/env python3
"""Fixed vs per-step cost of a cfg2 launch: kernel and wall time for 1..40
steps per launch, trace on and off (65 536 chains)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'scripts'))
from launch_probe import probe  # noqa: E402

if __name__ == '__main__':
  for trace in (True, False):
    for steps in (1, 2, 5, 10, 20, 40):
      probe('philox', False, steps, 20, None, trace=trace)
