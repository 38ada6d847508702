"""Engine: a spec (probayes_amd/spec.py) bound to one libpbhip engine/device.

Host-side precompute mirrors what the reference evaluates with NumPy/SciPy
once per model, so the device sees bit-identical constants:
  * log(scale) of every Normal (scipy norm.logpdf, _distn_infrastructure.py);
  * the mvn whitening matrix, log_pdet and rank of scipy's CovViaPSD
    (prob.py:349-358 -> multivariate_normal.pdf);
  * the CondCov tables coef / stdv / cdf limits (cond_cov.py:22-39).
Everything per chain-step runs in the HIP kernels; nothing here loops over
chains or steps.
"""
import atexit
import ctypes
import weakref

import numpy as np
import scipy.stats

from probayes_amd import _lib
from probayes_amd.spec import normalize_spec

_c = ctypes


def _dp(a):
  return a.ctypes.data_as(_c.POINTER(_c.c_double))


def _ip(a):
  return a.ctypes.data_as(_c.POINTER(_c.c_int32))


def _f64(a):
  return np.ascontiguousarray(a, dtype=np.float64)


def _i32(a):
  return np.ascontiguousarray(a, dtype=np.int32)


def condcov_tables(mean, cov, lo, hi):
  """CondCov.__init__ (cond_cov.py:22-39): per coordinate i the regression
  row Sigma_{i,-i} Sigma_{-i,-i}^{-1}, the Schur sd and the cdf limits of the
  bounds recentred on the unconditional mean (App. A-5)."""
  mean = np.atleast_1d(_f64(mean))
  cov = np.atleast_2d(_f64(cov))
  n = len(mean)
  lims = np.stack([_f64(lo), _f64(hi)], -1) - np.expand_dims(mean, -1)
  stdv = np.empty(n)
  coef = np.zeros((n, max(n - 1, 0)))
  for i in range(n):
    ll = np.delete(cov[:, i].reshape([n, 1]), i, axis=0)
    ru = np.delete(cov[i, :].reshape([1, n]), i, axis=1)
    sub = np.delete(np.delete(cov, i, axis=1), i, axis=0)
    row = ru.dot(np.linalg.inv(sub))
    coef[i] = row.reshape(-1)
    stdv[i] = np.sqrt(cov[i, i] - row.dot(ll).item())
  cdfs = np.array([scipy.stats.norm.cdf(lim, loc=0., scale=stdv[i])
                   for i, lim in enumerate(lims)])
  return coef, stdv, cdfs


def mvn_psd(mean, cov):
  """scipy multivariate_normal's CovViaPSD: (whitening U, rank*log(2pi) +
  log_pdet) exactly as scipy forms them (_multivariate.py _logpdf)."""
  mvn = scipy.stats.multivariate_normal(_f64(mean), _f64(cov))
  co = mvn.cov_object
  const = co.rank * np.log(2 * np.pi) + co.log_pdet
  return _f64(co._LP), float(const)


def unpack_stats(out, counts, d):
  """[world][3d+1][n_max] gather block (pbh_rccl_allgather_stats) -> the
  per-chain statistics of all ranks concatenated in rank (= global chain)
  order, padding columns dropped."""
  cols = [out[r, :, :counts[r]] for r in range(len(counts))]
  a = np.concatenate(cols, axis=1) if cols else np.empty((3 * d + 1, 0))
  return {'sum': a[:d].T.copy(), 'sumsq': a[d:2 * d].T.copy(),
          'n_acc': a[2 * d].astype(np.int64), 'ess': a[2 * d + 1:].T.copy(),
          'counts': np.asarray(counts, np.int64)}


# engines still open at interpreter exit are destroyed then (a resident
# sampling server is stopped and its chain state stored: no kernel outlives
# the process's last Python code)
_LIVE = weakref.WeakSet()


@atexit.register
def _close_live_engines():
  for eng in list(_LIVE):
    try:
      eng.close()
    except Exception:
      pass


def unpack_accept(acc, n):
  """Accept words [T, W] (uint64, bit c % 64 of word c // 64 = chain c) as
  u [N, T] uint8, C-contiguous.  The words are transposed first ([W, T]: 8
  bytes per 64 chains and record) and then unpacked along the chain axis --
  transposing the unpacked [T, N] bytes instead took ~2.8 s at 65 536 chains
  x 1 000 records (a strided read per byte)."""
  acc = np.ascontiguousarray(acc, np.uint64)
  count, W = acc.shape
  by = np.ascontiguousarray(
      np.ascontiguousarray(acc.T).view(np.uint8).reshape(W, count, 8).transpose(0, 2, 1))
  return np.unpackbits(by, axis=1, bitorder='little').reshape(W * 64, count)[:n]


class Engine:
  """One libpbhip engine on one device, running one lowered model."""

  def __init__(self, spec, device=0):
    self.spec = normalize_spec(spec)
    self.dim = self.spec['dim']
    self._h = _c.c_void_p()
    _lib.call('pbh_create', int(device), _c.byref(self._h))
    # the hot entry points, bound once (the timed run is two calls: a
    # getattr and c_int64 boxing per call were ~1 us of a 20-step run's ~35)
    lib = _lib.load()
    self._fn_run, self._fn_sync = lib.pbh_run, lib.pbh_sync
    self._fn_run_wait = lib.pbh_run_wait
    _LIVE.add(self)
    self.device = device
    self.n = 0
    self.chain_offset = 0
    self._rng = 'philox'
    self._set_model()
    if self.spec['proposal']['kind'] == 'gibbs':
      self._set_gibbs()
    else:
      self._set_proposal()

  # ---- model -------------------------------------------------------------
  def _set_model(self):
    s, d = self.spec, self.dim
    tg = s['target']
    m = _lib.PbhModel()
    m.dim = d
    m.target_kind = _lib.TARGET[tg['kind']]
    m.pscale = _lib.PSCALE[s['pscale']]
    m.scores = _lib.SCORES[s['scores']]
    keep = []

    def arr(a, conv=_f64):
      a = conv(a)
      keep.append(a)
      return a

    kind = tg['kind']
    if kind == 'diag_gauss':
      m.a, m.b = _dp(arr(tg['mu'])), _dp(arr(tg['sigma']))
      m.c = _dp(arr(np.log(_f64(tg['sigma']))))
      m.e = _dp(arr(1.0 / _f64(tg['sigma'])))
    elif kind == 'norm_iid':
      m.a = _dp(arr(tg['obs']))
      m.n = len(tg['obs'])
      m.i0, m.i1 = tg['loc'], tg['scale']
    elif kind == 'gmm':
      m.a, m.b = _dp(arr(tg['logw'])), _dp(arr(tg['mu']))
      m.c, m.e = _dp(arr(tg['sd'])), _dp(arr(np.log(_f64(tg['sd']))))
      m.n = len(tg['logw'])
    elif kind in ('norm_pdf',):
      m.a, m.b = _dp(arr(tg['loc'])), _dp(arr(tg['scale']))
    elif kind == 'uniform_pdf':
      m.a, m.b = _dp(arr(tg['lo'])), _dp(arr(tg['scale']))
    elif kind == 'mvn':
      U, const = mvn_psd(tg['mean'], tg['cov'])
      m.a, m.b = _dp(arr(tg['mean'])), _dp(arr(U))
      m.c = _dp(arr(np.array([const])))
    pr = s['prior']
    if pr is not None:
      m.has_prior = 1
      m.prior_lo, m.prior_hi = _dp(arr(pr['lo'])), _dp(arr(pr['hi']))
      m.prior_lo_incl = _ip(arr(pr['lo_incl'], _i32))
      m.prior_hi_incl = _ip(arr(pr['hi_incl'], _i32))
      m.prior_logp = pr['logp']
    m.ufun = _ip(arr(s['ufun'], _i32))
    tr = s['tran']
    m.tran_kind = _lib.TRAN[tr['kind']]
    m.tran_sym = 1 if tr['sym'] else 0
    if tr['kind'] == 'const':
      m.tran_value = tr['value']
    else:
      m.tran_scale = tr['scale']
      m.tran_offset = _dp(arr(tr['offset']))
      m.tran_order = _ip(arr(tr['order'], _i32))
    _lib.call('pbh_set_model', self._h, _c.byref(m))

  def _set_proposal(self):
    p, d = self.spec['proposal'], self.dim
    q = _lib.PbhProposal()
    q.kind = _lib.PROPOSAL[p['kind']]
    keep = []

    def arr(a, conv=_f64):
      a = conv(a)
      keep.append(a)
      return a

    if p['kind'] == 'gauss':
      q.loc, q.scale = _dp(arr(p['loc'])), _dp(arr(p['scale']))
      q.order = _ip(arr(p['order'], _i32))
    elif p['kind'] == 'sphere':
      q.delta = p['delta']
      q.lengths = _dp(arr(p['lengths']))
    elif p['kind'] == 'uniform':
      q.delta_vec = _dp(arr(p['delta']))
    elif p['kind'] == 'vardelta':
      q.delta_vec = _dp(arr(p['delta']))
      q.var_mode = _ip(arr(p['mode'], _i32))
    if p.get('vint') is not None:
      q.var_int = _ip(arr(p['vint'], _i32))
    b = p.get('bound')
    if b is not None:
      q.bound_on = _ip(arr(b['on'], _i32))
      q.bound_lo, q.bound_hi = _dp(arr(b['lo'])), _dp(arr(b['hi']))
      q.bound_xlo = _ip(arr(b['xlo'], _i32))
      q.bound_xhi = _ip(arr(b['xhi'], _i32))
    if p.get('tfun') is not None:
      q.tfun = _dp(arr(np.ascontiguousarray(p['tfun'], np.float64)))
    _lib.call('pbh_set_proposal', self._h, _c.byref(q))

  def _set_gibbs(self):
    p = self.spec['proposal']
    coef, stdv, cdfs = condcov_tables(p['mean'], p['cov'], p['lo'], p['hi'])
    keep = [_f64(p['mean']), _f64(coef), _f64(stdv), _f64(cdfs)]
    g = _lib.PbhGibbs()
    g.mean, g.coef, g.stdv, g.cdf = [_dp(a) for a in keep]
    g.tsteps = p['tsteps']
    _lib.call('pbh_set_gibbs', self._h, _c.byref(g))

  # ---- chains / randomness -------------------------------------------------
  def init_chains(self, init, chain_offset=0):
    """init [N, d] (or [d] broadcast to n chains via init_like)."""
    init = _f64(init).reshape(-1, self.dim)
    self.n = init.shape[0]
    _lib.call('pbh_init_chains', self._h, _c.c_int64(self.n),
              _c.c_int64(int(chain_offset)), _dp(init))
    self.chain_offset = int(chain_offset)

  def set_step(self, step):
    """Global step index of the first run step (the CondCov cycle phase,
    rf.py:446-452); right after init_chains."""
    _lib.call('pbh_set_step', self._h, _c.c_int64(int(step)))

  def set_rng(self, mode='philox', seed=0):
    _lib.call('pbh_set_rng', self._h, _lib.RNG[mode],
              _c.c_uint64(int(seed) & (2 ** 64 - 1)))
    self._rng = mode

  def stream_width(self):
    r = _c.c_int32()
    _lib.call('pbh_stream_width', self._h, _c.byref(r))
    return r.value

  def upload_replay(self, streams):
    """streams [T, R, N] in the reference's per-step consumption order."""
    streams = _f64(streams)
    T, R, N = streams.shape
    if N != self.n or R != self.stream_width():
      raise ValueError('replay stream shape {} does not match R={}, N={}'
                       .format(streams.shape, self.stream_width(), self.n))
    _lib.call('pbh_upload_replay', self._h, _c.c_int64(T), _dp(streams))

  def seed_legacy(self, seeds):
    """One NumPy legacy RandomState(seeds[c]) per chain, on the device."""
    seeds = np.ascontiguousarray(np.asarray(seeds).reshape(-1), dtype=np.int64)
    if seeds.size != self.n:
      raise ValueError('need {} seeds, got {}'.format(self.n, seeds.size))
    if np.any(seeds < 0) or np.any(seeds > 0xFFFFFFFF):
      raise ValueError('Seed must be between 0 and 2**32 - 1')
    s32 = np.ascontiguousarray(seeds.astype(np.uint32))
    _lib.call('pbh_legacy_seed', self._h,
              s32.ctypes.data_as(_c.POINTER(_c.c_uint32)))

  def legacy_replay(self, n_steps):
    """Fills the replay stream with the next n_steps rows of every chain's
    device RandomState (the reference's per-step draw order)."""
    _lib.call('pbh_legacy_replay', self._h, _c.c_int64(int(n_steps)))

  def reserve_replay(self, n_steps):
    """Sizes the replay stream buffer for n_steps rows (draws nothing): a
    later legacy_replay / upload_replay of at most that many rows allocates
    nothing.  Call it before filling the buffer."""
    _lib.call('pbh_reserve_replay', self._h, _c.c_int64(int(n_steps)))

  def get_replay(self, first, n_steps, draw=-1):
    """Rows of the current replay stream: [n, R, N], or [n, N] of one draw."""
    r = self.stream_width()
    shape = (n_steps, r, self.n) if draw < 0 else (n_steps, self.n)
    out = np.empty(shape, np.float64)
    _lib.call('pbh_get_replay', self._h, _c.c_int64(int(first)),
              _c.c_int64(int(n_steps)), int(draw), _dp(out))
    return out

  # ---- running -----------------------------------------------------------
  def alloc_trace(self, capacity, thin=1, debug=False, fill=True):
    """fill=False: no zero fill of the records (the next run writes every
    one of them: PBH_TRACE_NOFILL)."""
    flags = (1 if debug else 0) | (0 if fill else 0x100)
    _lib.call('pbh_alloc_trace', self._h, _c.c_int64(int(capacity)),
              int(thin), flags)
    self.debug = bool(debug)

  def run(self, n_steps, steps_per_launch=0, sync=True):
    # sync: one library call (pbh_run_wait) instead of pbh_run + pbh_sync
    fn = self._fn_run_wait if sync else self._fn_run
    rc = fn(self._h, int(n_steps), int(steps_per_launch))
    if rc:
      _lib.raise_status('pbh_run_wait' if sync else 'pbh_run', rc)

  def legacy_run(self, n_steps, steps_per_launch=0, sync=True):
    """legacy_replay(n) + run(n) in one kernel per launch (the draws go
    from each chain's device RandomState straight into the step): the same
    chains, trace and generator state; no replay rows are held afterwards."""
    _lib.call('pbh_legacy_run', self._h, _c.c_int64(int(n_steps)),
              int(steps_per_launch))
    if sync:
      self.sync()

  def set_record_threshold(self, on=True):
    """Keep each step's MH threshold t of the next legacy_run calls on the
    device (get_thresholds)."""
    _lib.call('pbh_set_record_threshold', self._h, 1 if on else 0)

  def get_thresholds(self, first, n_steps):
    """Thresholds of steps [first, first + n_steps) of the last legacy_run
    (set_record_threshold first): [n_steps, N]."""
    out = np.empty((int(n_steps), self.n), np.float64)
    _lib.call('pbh_get_thresholds', self._h, _c.c_int64(int(first)),
              _c.c_int64(int(n_steps)), _dp(out))
    return out

  def legacy_draws(self, n_steps, step0=0, kind='linreg', param=1.0):
    """The next n_steps draws of every chain's device RandomState, [n_steps,
    N]: kind 'linreg' -- standard_gamma(param) on steps (step0 + t) % 3 == 2,
    the legacy gauss otherwise (gibbs_linreg's cond_reg order); 'gauss' --
    the legacy gauss every step."""
    k = {'gauss': _lib.DRAWS_GAUSS, 'linreg': _lib.DRAWS_LINREG}[kind]
    out = np.empty((int(n_steps), self.n), np.float64)
    _lib.call('pbh_legacy_draws', self._h, _c.c_int64(int(n_steps)),
              _c.c_int64(int(step0)), k, _c.c_double(float(param)), _dp(out))
    return out

  def sync(self):
    rc = self._fn_sync(self._h)
    if rc:
      _lib.raise_status('pbh_sync', rc)

  def set_collect(self, moments=True):
    """moments=False: the kernels keep no running moments (no per-launch
    read-modify-write); trace_stats() reduces the recorded trace instead."""
    _lib.call('pbh_set_collect', self._h,
              _lib.COLLECT_MOMENTS if moments else 0)

  def last_run_ms(self):
    ms, nl = _c.c_double(), _c.c_int64()
    _lib.call('pbh_last_run_ms', self._h, _c.byref(ms), _c.byref(nl))
    return ms.value, nl.value

  def stop_server(self):
    """Stops the resident sampling server (PBH_SERVER=1) if it runs: the
    chain state is stored and the stream is idle afterwards."""
    _lib.call('pbh_server_stop', self._h)

  def server_stamps(self):
    """Per-workgroup (seq, t0, t1) of the server's last command (10 ns)."""
    cap = 4096
    q = np.zeros(cap, np.uint32)
    t0 = np.zeros(cap, np.uint64)
    t1 = np.zeros(cap, np.uint64)
    n = _c.c_int32()
    _lib.call('pbh_server_stamps', self._h, cap, q.ctypes.data_as(_lib._u32p),
              t0.ctypes.data_as(_lib._u64p), t1.ctypes.data_as(_lib._u64p),
              _c.byref(n))
    k = min(n.value, cap)
    return q[:k], t0[:k], t1[:k]

  def server_info(self):
    """{'active', 'commands', 'launches'} of the resident sampling server."""
    a, c, n = _c.c_int32(), _c.c_int64(), _c.c_int64()
    _lib.call('pbh_server_info', self._h, _c.byref(a), _c.byref(c), _c.byref(n))
    return {'active': bool(a.value), 'commands': c.value, 'launches': n.value}

  # ---- results -----------------------------------------------------------
  def state(self):
    x = np.empty((self.n, self.dim))
    lp = np.empty(self.n)
    _lib.call('pbh_get_state', self._h, _dp(x), _dp(lp))
    return x, lp

  def checkpoint(self):
    """Everything the chains need to continue exactly (pbh_get_checkpoint):
    x [N, d], lp [N], the global step, the step-1 flag, and the xoshiro
    generator state when that is the RNG."""
    x = np.empty((self.n, self.dim))
    lp = np.empty(self.n)
    step, hp = _c.c_int64(), _c.c_int32()
    xo = np.empty((8, self.n), np.uint32) if self._rng == 'xoshiro' else None
    _lib.call('pbh_get_checkpoint', self._h, _dp(x), _dp(lp), _c.byref(step),
              _c.byref(hp),
              None if xo is None else xo.ctypes.data_as(_lib._u32p))
    lx = np.empty((self.n, self.dim))
    valid = _c.c_int32()
    _lib.call('pbh_get_chain_logs', self._h, _dp(lx), _c.byref(valid))
    return {'x': x, 'lp': lp, 'step': step.value, 'has_pred': bool(hp.value),
            'xo': xo, 'mt': self._legacy_state(), 'chain_offset': self.chain_offset,
            'lx': lx if valid.value else None}

  def _legacy_state(self):
    """The device legacy streams' state (key, pos, has, gauss) or None."""
    words = _c.c_int64()
    _lib.call('pbh_legacy_state_words', self._h, _c.byref(words))
    if not words.value:
      return None
    key = np.empty((words.value, self.n), np.uint32)
    pos = np.empty(self.n, np.int32)
    has = np.empty(self.n, np.int32)
    gauss = np.empty(self.n)
    _lib.call('pbh_get_legacy_state', self._h, key.ctypes.data_as(_lib._u32p),
              pos.ctypes.data_as(_lib._i32p), has.ctypes.data_as(_lib._i32p),
              _dp(gauss))
    return {'key': key, 'pos': pos, 'has': has, 'gauss': gauss}

  def set_chains(self, x, lp, step, has_pred):
    """Replaces the chain state and step anywhere in a run; generator
    states continue (pbh_set_chains).  The trace and the replay rows are
    detached: alloc_trace (and upload_replay / legacy_replay) again."""
    x = np.ascontiguousarray(x, np.float64).reshape(self.n, self.dim)
    lp = np.ascontiguousarray(lp, np.float64).reshape(self.n)
    _lib.call('pbh_set_chains', self._h, _dp(x), _dp(lp), _c.c_int64(int(step)),
              1 if has_pred else 0)

  def restore(self, ck):
    """Resume from checkpoint() (after init_chains of the same N and set_rng
    with the same mode and seed, before alloc_trace)."""
    x = np.ascontiguousarray(ck['x'], np.float64)
    lp = np.ascontiguousarray(ck['lp'], np.float64)
    if x.shape != (self.n, self.dim) or lp.shape != (self.n,):
      raise ValueError('checkpoint shape does not match the engine')
    xo = ck.get('xo')
    xo = None if xo is None else np.ascontiguousarray(xo, np.uint32)
    if xo is not None and xo.size != 8 * self.n:   # [4 words][2 halves][N]
      raise ValueError('checkpoint xoshiro state has {} words, the engine needs '
                       '{}'.format(xo.size, 8 * self.n))
    mt = ck.get('mt')
    if mt is not None:
      # the C side copies words x N, N, N, N values from these arrays: a
      # checkpoint of the other legacy layout (PBH_LEGACY_DB) or of another
      # chain count would be read past its end
      words = _c.c_int64()
      _lib.call('pbh_legacy_state_words', self._h, _c.byref(words))
      want = {'key': (words.value, self.n), 'pos': (self.n,), 'has': (self.n,),
              'gauss': (self.n,)}
      layouts = {640: 'Mt4, its current chunked block (the default since round 6)',
                 2560: 'Mt4, four chunked blocks (rounds 4-5)',
                 1248: 'double-buffered window (PBH_LEGACY_K4=0, round 3)',
                 624: 'in-place state (PBH_LEGACY_DB=0, round 1)'}
      for k, shape in want.items():
        got = np.shape(mt[k])
        if got != shape:
          hint = ''
          if k == 'key' and len(got) == 2 and got[1] == self.n:
            hint = ('; the checkpoint holds the {} layout, this engine the {}: '
                    'restore it in an engine created with that layout\'s '
                    'environment'.format(
                        layouts.get(got[0], '{}-word'.format(got[0])),
                        layouts.get(words.value, '{}-word'.format(words.value))))
          raise ValueError('checkpoint legacy state {} has shape {}, this engine '
                           'needs {} (legacy layout words per chain: {}){}'.format(
                               k, got, shape, words.value, hint))
    _lib.call('pbh_restore', self._h, _dp(x), _dp(lp),
              _c.c_int64(int(ck['step'])), 1 if ck['has_pred'] else 0,
              None if xo is None else xo.ctypes.data_as(_lib._u32p))
    lx = ck.get('lx')
    if lx is not None:   # the production ufun logs (pbh_set_chain_logs)
      lx = np.ascontiguousarray(lx, np.float64)
      if lx.shape != (self.n, self.dim):
        raise ValueError('checkpoint ufun logs have shape {}, the engine needs {}'
                         .format(lx.shape, (self.n, self.dim)))
      _lib.call('pbh_set_chain_logs', self._h, _dp(lx))
    if mt is not None:   # device legacy streams continue where they were
      key = np.ascontiguousarray(mt['key'], np.uint32)
      pos = np.ascontiguousarray(mt['pos'], np.int32)
      has = np.ascontiguousarray(mt['has'], np.int32)
      gauss = np.ascontiguousarray(mt['gauss'], np.float64)
      _lib.call('pbh_set_legacy_state', self._h, key.ctypes.data_as(_lib._u32p),
                pos.ctypes.data_as(_lib._i32p), has.ctypes.data_as(_lib._i32p),
                _dp(gauss))

  def trace_len(self):
    r = _c.c_int64()
    _lib.call('pbh_trace_len', self._h, _c.byref(r))
    return r.value

  def trace(self, first=0, count=None, debug=None):
    """Recorded steps as chain-major arrays shaped like the golden fixtures:
    v_x [N, T, d], v_p [N, T], u [N, T] (uint8); with debug also p_x, p_p, s."""
    count = self.trace_len() - first if count is None else count
    n, d = self.n, self.dim
    W = (n + 63) // 64
    x = np.empty((count, d, n))
    lp = np.empty((count, n))
    acc = np.empty((count, W), np.uint64)
    debug = self.debug if debug is None else debug
    px = np.empty((count, d, n)) if debug else None
    pp = np.empty((count, n)) if debug else None
    sc = np.empty((count, n)) if debug else None
    nul = _c.POINTER(_c.c_double)()
    _lib.call('pbh_get_trace', self._h, _c.c_int64(first), _c.c_int64(count),
              _dp(x), _dp(lp), acc.ctypes.data_as(_c.POINTER(_c.c_uint64)),
              _dp(px) if debug else nul, _dp(pp) if debug else nul,
              _dp(sc) if debug else nul)
    out = {'v_x': x.transpose(2, 0, 1), 'v_p': lp.T, 'u': unpack_accept(acc, n)}
    if debug:
      out.update({'p_x': px.transpose(2, 0, 1), 'p_p': pp.T, 's': sc.T})
    return out

  def moments(self):
    n, d = self.n, self.dim
    s = np.empty((d, n))
    q = np.empty((d, n))
    na = np.empty(n, np.int64)
    steps = _c.c_int64()
    _lib.call('pbh_get_moments', self._h, _dp(s), _dp(q),
              na.ctypes.data_as(_c.POINTER(_c.c_int64)), _c.byref(steps))
    return {'sum': s.T.copy(), 'sumsq': q.T.copy(), 'n_acc': na,
            'n_steps': steps.value}

  def trace_stats(self, first=0, count=None):
    """Per-chain sum / sumsq / n_acc of trace records [first, first +
    count), reduced on the device (also replaces the engine's moments)."""
    count = self.trace_len() - first if count is None else count
    n, d = self.n, self.dim
    s = np.empty((d, n))
    q = np.empty((d, n))
    na = np.empty(n, np.int64)
    _lib.call('pbh_trace_stats', self._h, _c.c_int64(int(first)),
              _c.c_int64(int(count)), _dp(s), _dp(q),
              na.ctypes.data_as(_c.POINTER(_c.c_int64)))
    return {'sum': s.T.copy(), 'sumsq': q.T.copy(), 'n_acc': na,
            'n_steps': int(count)}

  def reset_moments(self):
    _lib.call('pbh_reset_moments', self._h)

  # ---- RCCL ---------------------------------------------------------------
  @staticmethod
  def rccl_unique_id():
    buf = (_c.c_uint8 * 128)()
    _lib.call('pbh_rccl_unique_id', buf)
    return bytes(buf)

  def rccl_init(self, rank, world, uid):
    buf = (_c.c_uint8 * 128).from_buffer_copy(uid)
    _lib.call('pbh_rccl_init', self._h, int(rank), int(world), buf)
    self.world = int(world)

  def rccl_allgather_stats(self):
    """The one RCCL all-gather: every rank's per-chain statistics, in
    global chain order (ranks hold contiguous blocks, dist.shard).  Returns
    {'sum': [N, d], 'sumsq': [N, d], 'n_acc': [N], 'ess': [N, d],
    'counts': [world]}; ess is NaN for a rank that never ran trace_ess."""
    d = self.dim
    nm = _c.c_int64()
    _lib.call('pbh_rccl_max_chains', self._h, _c.byref(nm))
    out = np.empty((self.world, 3 * d + 1, nm.value))
    counts = np.empty(self.world, np.int64)
    _lib.call('pbh_rccl_allgather_stats', self._h, _dp(out),
              counts.ctypes.data_as(_c.POINTER(_c.c_int64)))
    return unpack_stats(out, counts, d)

  def trace_ess(self, first=0, count=None):
    """Per-chain, per-dim initial-positive-sequence ESS of trace records
    [first, first + count), computed on the device: [N, d]."""
    count = self.trace_len() - first if count is None else count
    out = np.empty((self.dim, self.n))
    _lib.call('pbh_trace_ess', self._h, _c.c_int64(int(first)),
              _c.c_int64(int(count)), _dp(out))
    return out.T   # a [N, d] view of the [d][N] result (no 2-D transpose copy)

  def trace_ess_total(self, first=0, count=None):
    """Per dim, the sum over chains of trace_ess (reduced on the device):
    [d]."""
    count = self.trace_len() - first if count is None else count
    out = np.empty(self.dim)
    _lib.call('pbh_trace_ess_total', self._h, _c.c_int64(int(first)),
              _c.c_int64(int(count)), _dp(out))
    return out

  def trace_expectation(self, first=0, count=None, exponent=None):
    """PD.expectation (pd.py:373-405) of the summary of trace records
    [first, first + count), computed on the device: [N, d] of
    sum p v^exponent / sum p with p the recorded prob rescaled to linear."""
    count = self.trace_len() - first if count is None else count
    out = np.empty((self.dim, self.n))
    _lib.call('pbh_trace_expectation', self._h, _c.c_int64(int(first)),
              _c.c_int64(int(count)), _c.c_double(float(exponent or 0.)),
              _dp(out))
    return out.T.copy()

  def rccl_allreduce_max(self, value):
    v = _c.c_double(float(value))
    _lib.call('pbh_rccl_allreduce_max', self._h, _c.byref(v))
    return v.value

  @staticmethod
  def cache_release():
    """Frees the device buffers and streams destroyed engines left in the
    library's resource cache (pbh_cache_release)."""
    _lib.call('pbh_cache_release')

  @staticmethod
  def cache_info():
    """(idle bytes, hits, misses) of the library's resource cache."""
    v = [_c.c_int64() for _ in range(3)]
    _lib.call('pbh_cache_info', *[_c.byref(x) for x in v])
    return tuple(x.value for x in v)

  def close(self):
    if getattr(self, '_h', None) is not None and self._h.value:
      _lib.load().pbh_destroy(self._h)
      self._h = _c.c_void_p()

  def __del__(self):
    try:
      self.close()
    except Exception:
      pass

  def __enter__(self):
    return self

  def __exit__(self, *exc):
    self.close()
