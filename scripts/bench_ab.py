#!/usr/bin/env python3
"""A/B of two builds of libpbhip on one box: runs bench.py's main with
probayes_amd._lib pointed at the given library (argv[1]); the remaining
arguments go to bench.py."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import probayes_amd._lib as L  # noqa: E402

L.LIB_PATH = os.path.join(ROOT, sys.argv[1])
sys.argv = ['bench.py'] + sys.argv[2:]
runpy.run_path(os.path.join(ROOT, 'bench.py'), run_name='__main__')
