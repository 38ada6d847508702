"""ctypes binding of libpbhip.so (include/pbhip.h).

This is the reference-side binding INTEGRATION.md describes: plain ctypes over
the C-ABI, no torch types.  The library is loaded from the package directory
(built in-tree by `make -C probayes_amd/csrc`) or from $PBHIP_LIB.  There is no
fallback: if the library is missing every engine call raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('PBHIP_LIB', os.path.join(_HERE, 'libpbhip.so'))

ABI_VERSION = 6
DRAWS_GAUSS, DRAWS_LINREG = 0, 1   # enum pbh_draws
MAX_DIM = 32

# enums (pbhip.h)
TARGET = {'diag_gauss': 1, 'norm_iid': 2, 'gmm': 3, 'norm_pdf': 4,
          'uniform_pdf': 5, 'mvn': 6}
PSCALE = {'log': 0, 'lin': 1}
SCORES = {'hastings': 1, 'metropolis': 2, 'gibbs': 3}
TRAN = {'const': 1, 'gauss_pdf': 2}
PROPOSAL = {'gauss': 1, 'sphere': 2, 'uniform': 3, 'gibbs': 4, 'vardelta': 5}
# enum pbh_var_delta
VAR_FIXED, VAR_POLARITY, VAR_UNIFORM, VAR_RANDINT = 0, 1, 2, 3
RNG = {'replay': 0, 'philox': 1, 'philox_f64': 2, 'xoshiro': 3,
       'philox_fp32': 4}
COLLECT_MOMENTS = 1

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int32)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_i32p = ctypes.POINTER(ctypes.c_int32)
_i64p = ctypes.POINTER(ctypes.c_int64)
_u64p = ctypes.POINTER(ctypes.c_uint64)


class PbhModel(ctypes.Structure):
  _fields_ = [
      ('dim', ctypes.c_int32), ('target_kind', ctypes.c_int32),
      ('pscale', ctypes.c_int32), ('scores', ctypes.c_int32),
      ('a', _dp), ('b', _dp), ('c', _dp), ('e', _dp), ('perm', _ip),
      ('n', ctypes.c_int64), ('i0', ctypes.c_int32), ('i1', ctypes.c_int32),
      ('has_prior', ctypes.c_int32),
      ('prior_lo', _dp), ('prior_hi', _dp),
      ('prior_lo_incl', _ip), ('prior_hi_incl', _ip),
      ('prior_logp', ctypes.c_double),
      ('ufun', _ip),
      ('tran_kind', ctypes.c_int32), ('tran_sym', ctypes.c_int32),
      ('tran_value', ctypes.c_double), ('tran_scale', ctypes.c_double),
      ('tran_offset', _dp), ('tran_order', _ip),
  ]


class PbhProposal(ctypes.Structure):
  _fields_ = [
      ('kind', ctypes.c_int32), ('loc', _dp), ('scale', _dp),
      ('order', _ip), ('delta', ctypes.c_double), ('lengths', _dp),
      ('delta_vec', _dp), ('tfun', _dp), ('var_mode', _ip), ('var_int', _ip),
      ('bound_on', _ip), ('bound_lo', _dp), ('bound_hi', _dp),
      ('bound_xlo', _ip), ('bound_xhi', _ip),
  ]


class PbhGibbs(ctypes.Structure):
  _fields_ = [('mean', _dp), ('coef', _dp), ('stdv', _dp), ('cdf', _dp),
              ('tsteps', ctypes.c_int32)]


# name -> (restype, argtypes); every symbol include/pbhip.h declares.
SIGNATURES = {
    'pbh_last_error': (ctypes.c_char_p, []),
    'pbh_abi_version': (ctypes.c_int, []),
    'pbh_device_count': (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    'pbh_create': (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    'pbh_destroy': (ctypes.c_int, [ctypes.c_void_p]),
    'pbh_cache_release': (ctypes.c_int, []),
    'pbh_cache_info': (ctypes.c_int, [ctypes.POINTER(ctypes.c_int64)] * 3),
    'pbh_set_model': (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(PbhModel)]),
    'pbh_set_proposal': (ctypes.c_int, [ctypes.c_void_p,
                                        ctypes.POINTER(PbhProposal)]),
    'pbh_set_gibbs': (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(PbhGibbs)]),
    'pbh_init_chains': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64,
                                       ctypes.c_int64, _dp]),
    'pbh_set_step': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
    'pbh_set_rng': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32,
                                   ctypes.c_uint64]),
    'pbh_upload_replay': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, _dp]),
    'pbh_stream_width': (ctypes.c_int, [ctypes.c_void_p, _ip]),
    'pbh_legacy_seed': (ctypes.c_int, [ctypes.c_void_p, _u32p]),
    'pbh_legacy_replay': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
    'pbh_reserve_replay': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
    'pbh_legacy_run': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32]),
    'pbh_set_record_threshold': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32]),
    'pbh_get_thresholds': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.c_int64, _dp]),
    'pbh_legacy_draws': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                        ctypes.c_int32, ctypes.c_double, _dp]),
    'pbh_get_replay': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64,
                                      ctypes.c_int64, ctypes.c_int32, _dp]),
    'pbh_alloc_trace': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64,
                                       ctypes.c_int32, ctypes.c_int32]),
    'pbh_run': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32]),
    'pbh_sync': (ctypes.c_int, [ctypes.c_void_p]),
    'pbh_run_wait': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32]),
    'pbh_trace_ess_total': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64,
                                           ctypes.c_int64, _dp]),
    'pbh_set_collect': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32]),
    'pbh_last_run_ms': (ctypes.c_int, [ctypes.c_void_p, _dp, _i64p]),
    'pbh_server_stop': (ctypes.c_int, [ctypes.c_void_p]),
    'pbh_get_chain_logs': (ctypes.c_int, [ctypes.c_void_p, _dp, _ip]),
    'pbh_set_chain_logs': (ctypes.c_int, [ctypes.c_void_p, _dp]),
    'pbh_server_info': (ctypes.c_int, [ctypes.c_void_p, _ip, _i64p, _i64p]),
    'pbh_server_stamps': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, _u32p,
                                         _u64p, _u64p, _ip]),
    'pbh_get_state': (ctypes.c_int, [ctypes.c_void_p, _dp, _dp]),
    'pbh_trace_len': (ctypes.c_int, [ctypes.c_void_p, _i64p]),
    'pbh_get_trace': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64,
                                     ctypes.c_int64, _dp, _dp, _u64p, _dp, _dp,
                                     _dp]),
    'pbh_get_moments': (ctypes.c_int, [ctypes.c_void_p, _dp, _dp, _i64p, _i64p]),
    'pbh_reset_moments': (ctypes.c_int, [ctypes.c_void_p]),
    'pbh_trace_stats': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64,
                                       ctypes.c_int64, _dp, _dp, _i64p]),
    'pbh_rccl_unique_id': (ctypes.c_int, [_u8p]),
    'pbh_rccl_init': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32,
                                     ctypes.c_int32, _u8p]),
    'pbh_rccl_max_chains': (ctypes.c_int, [ctypes.c_void_p, _i64p]),
    'pbh_rccl_allgather_stats': (ctypes.c_int, [ctypes.c_void_p, _dp, _i64p]),
    'pbh_get_checkpoint': (ctypes.c_int, [ctypes.c_void_p, _dp, _dp,
                                          ctypes.POINTER(ctypes.c_int64),
                                          ctypes.POINTER(ctypes.c_int32),
                                          _u32p]),
    'pbh_restore': (ctypes.c_int, [ctypes.c_void_p, _dp, _dp, ctypes.c_int64,
                                   ctypes.c_int32, _u32p]),
    'pbh_set_chains': (ctypes.c_int, [ctypes.c_void_p, _dp, _dp, ctypes.c_int64,
                                      ctypes.c_int32]),
    'pbh_legacy_state_words': (ctypes.c_int, [ctypes.c_void_p,
                                              ctypes.POINTER(ctypes.c_int64)]),
    'pbh_get_legacy_state': (ctypes.c_int, [ctypes.c_void_p, _u32p, _i32p, _i32p,
                                            _dp]),
    'pbh_set_legacy_state': (ctypes.c_int, [ctypes.c_void_p, _u32p, _i32p, _i32p,
                                            _dp]),
    'pbh_trace_expectation': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64,
                                             ctypes.c_int64, ctypes.c_double,
                                             _dp]),
    'pbh_trace_ess': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64,
                                     ctypes.c_int64, _dp]),
    'pbh_rccl_allreduce_max': (ctypes.c_int, [ctypes.c_void_p, _dp]),
    'pbh_rccl_destroy': (ctypes.c_int, [ctypes.c_void_p]),
    'pbh_check_accept': (ctypes.c_int, [ctypes.c_int, ctypes.c_int64, _dp, _dp,
                                        _u32p, _u32p, ctypes.c_int32, _u8p]),
    'pbh_check_normals': (ctypes.c_int, [ctypes.c_int, ctypes.c_int64, _u32p,
                                         _dp, _dp]),
    'pbh_check_normals64': (ctypes.c_int, [ctypes.c_int, ctypes.c_int64, _u32p,
                                           _dp, _dp]),
    'pbh_bm64_tables': (ctypes.c_int, [_dp]),
    'pbh_bool_perm_freq': (ctypes.c_int, [ctypes.c_int, ctypes.c_int64,
                                          ctypes.c_int32,
                                          ctypes.POINTER(ctypes.c_uint8),
                                          ctypes.POINTER(ctypes.c_int64),
                                          ctypes.c_int32,
                                          ctypes.POINTER(ctypes.c_double)]),
    'pbh_linreg_gibbs': (ctypes.c_int, [
        ctypes.c_int, ctypes.c_int64, _dp, _dp, _dp, _dp, ctypes.c_int64,
        ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, _dp, ctypes.c_int32,
        ctypes.c_uint64, _dp, _dp, _dp, _dp, _dp, ctypes.c_int32, _dp]),
}


class PbhError(RuntimeError):
  """A libpbhip status != 0 (message from pbh_last_error)."""

  def __init__(self, fn, code, msg):
    super().__init__('{} -> {}: {}'.format(fn, code, msg))
    self.code = code


_LIB = None


def load():
  """Loads libpbhip.so once; raises (loudly) if it is missing."""
  global _LIB
  if _LIB is not None:
    return _LIB
  if not os.path.exists(LIB_PATH):
    raise OSError('libpbhip.so not found at {} -- build it with '
                  '`make -C probayes_amd/csrc` (or __graft_entry__.build())'
                  .format(LIB_PATH))
  lib = ctypes.CDLL(LIB_PATH)
  for name, (res, args) in SIGNATURES.items():
    fn = getattr(lib, name)
    fn.restype = res
    fn.argtypes = args
  if lib.pbh_abi_version() != ABI_VERSION:
    raise OSError('libpbhip ABI {} != {}'.format(lib.pbh_abi_version(),
                                                  ABI_VERSION))
  _LIB = lib
  return lib


def raise_status(name, rc):
  raise PbhError(name, rc, load().pbh_last_error().decode())


def call(name, *args):
  lib = load()
  rc = getattr(lib, name)(*args)
  if rc != 0:
    raise_status(name, rc)
  return rc
