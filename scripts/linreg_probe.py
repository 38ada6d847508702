"""Times the linreg Gibbs kernel (pbh_linreg_gibbs) on one GPU: 65 536 (and
262 144) chains x 1 000 steps per launch, each RNG mode; prints one JSON line per mode."""
import json
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from probayes_amd import linreg

rs = np.random.RandomState(321)
x = rs.normal(0, 1, size=60)
y = rs.normal(1.5 * x - 1., 0.5)
t = 1000
for rng, n in (('philox', 65536), ('philox', 262144), ('philox_pair', 65536),
               ('philox_f64', 65536), ('replay', 65536)):
  os.environ['PBH_LINREG_PAIR'] = '1' if rng == 'philox_pair' else '0'
  init = np.tile([-0.9, 1.4, 0.6], (n, 1))
  rand = np.abs(rs.normal(size=(t, n))) + 0.5 if rng == 'replay' else None
  o = linreg.run(x, y, init, t, rng=rng.replace('_pair', ''), seed=1, rand=rand, reps=5,
                 trace=False)
  ms = o['ms']
  B = 4 * 8 + (8 if rng == 'replay' else 0)   # trace 3 x + lp (+ draw read)
  print(json.dumps({'kernel': 'linreg_gibbs', 'rng': rng, 'chains': n,
                    'steps': t, 'ms': ms, 'steps_per_s': n * t / ms * 1e3,
                    'GB_per_s': n * t * B / ms / 1e6}), flush=True)
