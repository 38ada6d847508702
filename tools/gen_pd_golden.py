"""Golden vectors for the summary-PD operations: runs the
REFERENCE probayes in this container only (recipe: tools/gen_golden.py) and
records, for MH summaries of a 1-variable and a 2-variable model, the summary
values/probabilities together with the reference's own
PD.expectation (pd.py:373-405), PD.sorted (pd.py:463-493) and
PD.quantile (pd.py:408-460) outputs, and the exception types
PD.conditionalise (pd.py:214-295) raises on such summaries.  Output: tests/golden/pd_ops.npz.
Nothing in tests/, bench.py or __graft_entry__ imports this script.
"""
import json
import os

import numpy as np
import scipy.stats

import probayes as pb

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   'tests', 'golden', 'pd_ops.npz')
QS = [0.1, 0.5, 0.9]


def summary_1d(seed, steps):
  np.random.seed(seed)
  x = pb.RV('x', vtype=float, vset=(-10., 10.))
  process = pb.SP(pb.RF(x))
  def lp(**kw):   # a def: the reference calls argument-free lambdas bare
    return scipy.stats.norm.logpdf(kw['x'], 1., 2.)
  process.set_prob(lp, pscale='log')
  process.set_tran(lambda **kw: 1.)
  process.set_delta(lambda: process.Delta(x=scipy.stats.norm.rvs(scale=0.5)))
  process.set_scores('hastings')
  process.set_update('metropolis')
  return process([s for s in process.sampler({'x': 0.}, stop=steps)]).v


def summary_2d(seed, steps):
  np.random.seed(seed)
  x = pb.RV('x', vtype=float, vset=(-10., 10.))
  y = pb.RV('y', vtype=float, vset=(-10., 10.))
  process = pb.SP(x & y)
  def lp(**kw):
    return (scipy.stats.norm.logpdf(kw['x'], 1., 2.) +
            scipy.stats.norm.logpdf(kw['y'], -1., .5))
  process.set_prob(lp, pscale='log')
  process.set_tran(lambda **kw: 1.)
  process.set_delta(lambda: process.Delta(x=scipy.stats.norm.rvs(scale=0.5),
                                          y=scipy.stats.norm.rvs(scale=0.3)))
  process.set_scores('hastings')
  process.set_update('metropolis')
  return process([s for s in process.sampler({'x': 0., 'y': 0.},
                                             stop=steps)]).v


def main():
  out, meta = {}, {'qs': QS, 'cases': []}
  for name, fn, seed, steps in [('a', summary_1d, 5, 60),
                                ('b', summary_2d, 9, 80)]:
    v = fn(seed, steps)
    keys = list(v.keys())
    meta['cases'].append({'name': name, 'keys': keys})
    for k in keys:
      out['{}_val_{}'.format(name, k)] = np.asarray(v[k], float)
      out['{}_exp_{}'.format(name, k)] = float(v.expectation()[k])
      out['{}_exp2_{}'.format(name, k)] = float(v.expectation(exponent=2)[k])
    out['{}_prob'.format(name)] = np.asarray(v.prob, float)
    srt = v.sorted(keys[0])
    for k in keys:
      out['{}_sorted_{}'.format(name, k)] = np.asarray(srt[k], float)
    out['{}_sorted_prob'.format(name)] = np.asarray(srt.prob, float)
    quants = srt.quantile(QS)
    for k in keys:
      qv = [qq[k] for qq in quants]
      # unsorted keys come back as {size}
      out['{}_quant_{}'.format(name, k)] = np.array(
          [float(next(iter(z))) if isinstance(z, set) else float(z) for z in qv])
      out['{}_quant_isset_{}'.format(name, k)] = np.array(
          [isinstance(z, set) for z in qv])
    # conditionalise (pd.py:214-295) on a summary: record what the reference
    # raises for all keys and for a strict subset
    errs = []
    for ks in [keys] + ([keys[:1]] if len(keys) > 1 else []):
      try:
        v.conditionalise(ks)
        errs.append('')
      except Exception as e:  # pylint: disable=broad-except
        errs.append(type(e).__name__)
    meta['cases'][-1]['cond_errors'] = errs
    uq = v.quantile(0.5)
    out['{}_unsorted_quant_isset'.format(name)] = np.array(
        [isinstance(uq[k], set) for k in keys])
  out['meta'] = np.array(json.dumps(meta))
  np.savez(OUT, **out)
  print('wrote', OUT, sorted(out))


if __name__ == '__main__':
  main()
