"""The resident sampling server (PBH_SERVER=1, pbh_server_*): the FULL
lane-pair kernel stays resident and each eligible pbh_run is a command.  The
chains must be bit-for-bit those of ordinary launches (the same kernel body,
the same words), and the server must stop, restart, leave on its own when
idle, and never outlive the process."""
import os
import subprocess
import sys
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu

N = 8192   # 32 eight-wave workgroups


def _engine(monkeypatch, server, idle_ms=None):
  import bench
  from probayes_amd import Engine
  monkeypatch.setenv('PBH_SERVER', '1' if server else '0')
  if idle_ms is not None:
    monkeypatch.setenv('PBH_SERVER_IDLE_MS', str(idle_ms))
  eng = Engine(bench.cfg2_spec())
  x0 = np.random.RandomState(5).normal(size=(N, bench.D))
  eng.init_chains(x0)
  eng.set_rng('philox', seed=31)
  eng.set_collect(moments=False)
  eng.alloc_trace(400, 1)
  return eng


def _runs(eng, plan, between=None):
  for i, k in enumerate(plan):
    eng.run(k, steps_per_launch=k)
    if between:
      between(i, eng)


PLAN = [1, 1, 1, 1, 20, 7, 1, 2, 3, 64, 65, 1, 100]   # odd / even starts and ends


def test_server_commands_equal_launches(monkeypatch):
  ref = _engine(monkeypatch, False)
  _runs(ref, PLAN)
  tr_ref, st_ref = ref.trace(), ref.state()
  ref.close()
  eng = _engine(monkeypatch, True)
  _runs(eng, PLAN)
  info = eng.server_info()
  assert info['commands'] == len(PLAN) - 1 and info['launches'] == 1, info
  tr, st = eng.trace(), eng.state()     # get_trace stops the server first
  assert not eng.server_info()['active']
  eng.close()
  for k in ('v_x', 'v_p', 'u'):
    assert np.array_equal(tr[k], tr_ref[k]), k
  assert np.array_equal(st[0], st_ref[0]) and np.array_equal(st[1], st_ref[1])
  assert 0.05 < tr['u'].mean() < 0.95


def test_server_stop_start_restart_and_entry_points(monkeypatch):
  """stop_server, an entry point between commands (trace_stats stops it),
  and the next eligible run relaunching it: the same chains as launches."""
  def between(i, eng):
    if i == 4:
      eng.stop_server()
      assert not eng.server_info()['active']
    if i == 8:
      eng.trace_stats(0, 10)
  ref = _engine(monkeypatch, False)
  _runs(ref, PLAN, between)
  tr_ref = ref.trace()
  ref.close()
  eng = _engine(monkeypatch, True)
  _runs(eng, PLAN, between)
  info = eng.server_info()
  assert info['launches'] == 3, info
  tr = eng.trace()
  eng.close()
  for k in ('v_x', 'v_p', 'u'):
    assert np.array_equal(tr[k], tr_ref[k]), k


def test_server_leaves_when_idle_and_is_relaunched(monkeypatch):
  eng = _engine(monkeypatch, True, idle_ms=40)
  eng.run(1)
  eng.run(20)
  assert eng.server_info()['active']
  time.sleep(0.3)                        # > the 40 ms idle exit
  assert not eng.server_info()['active']  # the kernel ended by itself
  eng.run(20)                            # relaunched, not a lost command
  info = eng.server_info()
  assert info['launches'] == 2 and info['commands'] == 2, info
  tr = eng.trace()
  eng.close()
  ref = _engine(monkeypatch, False)
  ref.run(1)
  ref.run(20)
  ref.run(20)
  tr_ref = ref.trace()
  ref.close()
  for k in ('v_x', 'v_p', 'u'):
    assert np.array_equal(tr[k], tr_ref[k]), k


def test_server_idle_measured_from_the_submit(monkeypatch):
  """a sync long after a command must not restart the host's
  idle clock -- the kernel's workgroups start theirs at the command's
  completion.  run(sync=False), 0.7 idle later sync, 0.4 idle later run: the
  kernel has left by then (1.1 idle after the completion), so the run must
  relaunch it rather than command a server that is gone."""
  idle = 200
  eng = _engine(monkeypatch, True, idle_ms=idle)
  eng.run(1)
  eng.run(20, sync=False)
  time.sleep(0.7 * idle / 1e3)
  eng.sync()
  time.sleep(0.4 * idle / 1e3)
  eng.run(20)
  info = eng.server_info()
  assert info['launches'] == 2 and info['commands'] == 2, info
  tr = eng.trace()
  eng.close()
  ref = _engine(monkeypatch, False)
  ref.run(1)
  ref.run(20)
  ref.run(20)
  tr_ref = ref.trace()
  ref.close()
  for k in ('v_x', 'v_p', 'u'):
    assert np.array_equal(tr[k], tr_ref[k]), k


def test_server_command_time_and_sync(monkeypatch):
  eng = _engine(monkeypatch, True)
  eng.run(1)
  eng.run(2)
  t0 = time.perf_counter()
  eng.run(100, sync=False)
  eng.sync()
  wall_ms = (time.perf_counter() - t0) * 1e3
  ms, launches = eng.last_run_ms()
  assert launches == 1 and 0 < ms < wall_ms, (ms, wall_ms)
  eng.close()


EXIT_SCRIPT = r'''
import os, sys
sys.path.insert(0, {root!r})
os.environ['PBH_SERVER'] = '1'
os.environ['PBH_SERVER_IDLE_MS'] = '60000'
import numpy as np, bench
from probayes_amd import Engine
eng = Engine(bench.cfg2_spec())
eng.init_chains(np.zeros(({n}, bench.D)))
eng.set_rng('philox', seed=1)
eng.set_collect(moments=False)
eng.alloc_trace(50, 1)
eng.run(1)
eng.run(20)
assert eng.server_info()['active']
print('LEAVING', flush=True)
# no close(): the interpreter's exit must stop the server
'''


def test_server_does_not_outlive_the_process(tmp_path):
  script = tmp_path / 'leave.py'
  script.write_text(EXIT_SCRIPT.format(root=ROOT, n=N))
  t0 = time.perf_counter()
  p = subprocess.run([sys.executable, str(script)], capture_output=True, text=True,
                     timeout=90)
  el = time.perf_counter() - t0
  assert p.returncode == 0 and 'LEAVING' in p.stdout, p.stdout + p.stderr
  assert el < 30   # the atexit stop, not the kernel's 60 s idle exit
