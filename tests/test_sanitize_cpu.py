"""Sanitizer run of the conv launch planners (SURVEY §5 race detection / sanitizers): the host code of
``csrc/conv.hip`` built with AddressSanitizer + UBSan (host side only -- GPU ASan / xnack builds are
not available on this pool) and ``conv_plan_selfcheck`` run over ~20k layer geometries on the CPU:
LDS budgets, staging-register capacities, tile coverage, cursor steps, weight-row padding, grid sizes."""
import hashlib
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which('hipcc') is None and not os.path.exists('/opt/rocm/bin/hipcc'),
                    reason='hipcc not available')
def test_conv_planner_under_asan_ubsan():
    srcs = [os.path.join(ROOT, 'csrc', f) for f in ('conv.hip', 'conv_bwd.hip', 'common.h', 'launchers.h')]
    srcs += [os.path.join(ROOT, 'tools', 'sanitize', f) for f in ('plan_check.cpp', 'run.sh')]
    h = hashlib.sha1(b''.join(open(f, 'rb').read() for f in srcs)).hexdigest()[:12]
    exe = f'/tmp/msp_plan_check_{h}'
    if os.path.exists(exe):   # built for this exact source: just run it (sanitizers stay compiled in)
        env = dict(os.environ, ASAN_OPTIONS='detect_leaks=0:abort_on_error=1', UBSAN_OPTIONS='print_stacktrace=1')
        r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    else:
        r = subprocess.run(['bash', os.path.join(ROOT, 'tools', 'sanitize', 'run.sh'), exe], capture_output=True,
                           text=True, timeout=1200)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert 'PLAN_CHECK_OK' in out and '0 violations' in out, out[-4000:]
    assert 'ERROR: AddressSanitizer' not in out and 'runtime error' not in out, out[-4000:]
