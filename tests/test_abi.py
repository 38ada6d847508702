"""CPU checks of the C-ABI library: it loads (no GPU needed), exports every
function include/pbhip.h declares, and reports errors through status codes."""
import ctypes
import os
import re

import pytest

from probayes_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
  src = open(os.path.join(ROOT, 'include', 'pbhip.h')).read()
  src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
  return sorted(set(re.findall(r'\b(pbh_[a-z0-9_]+)\s*\(', src)))


def test_library_exports_every_declared_symbol():
  lib = _lib.load()
  names = _header_functions()
  assert len(names) >= 25
  for name in names:
    assert hasattr(lib, name), name
  assert set(names) == set(_lib.SIGNATURES), \
      set(names) ^ set(_lib.SIGNATURES)


def test_abi_version_and_error_reporting():
  lib = _lib.load()
  assert lib.pbh_abi_version() == _lib.ABI_VERSION
  eng = ctypes.c_void_p()
  rc = lib.pbh_create(-1, ctypes.byref(eng))
  assert rc != 0
  assert lib.pbh_last_error()
  assert lib.pbh_run(None, 1, 0) == -1          # NULL engine -> PBH_ERR_ARG
  assert b'engine' in lib.pbh_last_error()
  with pytest.raises(_lib.PbhError):
    _lib.call('pbh_sync', None)


def test_library_targets_gfx950():
  so = open(_lib.LIB_PATH, 'rb').read()
  assert b'gfx950' in so
