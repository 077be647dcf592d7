#!/usr/bin/env python3
"""Build the HIP extension in-tree for gfx950 (no hipify, no torch JIT cache).

Every ``csrc/*.hip`` kernel file is compiled by ``hipcc --offload-arch=gfx950`` into an object with
a plain C++ launch API (``launchers.h``); ``bindings.cpp`` adapts torch tensors; the result is linked
into ``medical_segmentation_pytorch_amd/_C.so`` against the HIP runtime that ships with torch (one
runtime per process).  Uses ninja for incremental, parallel builds.

    python csrc/build.py [--jobs N] [--verbose]
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, 'medical_segmentation_pytorch_amd')
# MSP_BUILD_VARIANT=<name>: a side build (e.g. with extra -D flags in MSP_BUILD_DEFINES) written to
# build/<name>/_C.so and loaded instead of the product extension when env MSP_C_SO points at it
VARIANT = os.environ.get('MSP_BUILD_VARIANT', '')
BUILD = os.path.join(ROOT, 'build', 'csrc' + (f'_{VARIANT}' if VARIANT else ''))
ARCH = os.environ.get('PYTORCH_ROCM_ARCH', 'gfx950').split(';')[0]
ROCM = os.environ.get('ROCM_PATH', '/opt/rocm')


def torch_paths():
    import torch
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, 'include'), os.path.join(tdir, 'include', 'torch', 'csrc', 'api', 'include')]
    return tdir, inc, int(torch._C._GLIBCXX_USE_CXX11_ABI)


def write_ninja(jobs):
    tdir, tinc, abi = torch_paths()
    pyinc = sysconfig.get_paths()['include']
    import pybind11
    hipcc = shutil.which('hipcc') or os.path.join(ROCM, 'bin', 'hipcc')
    kernels = sorted(f for f in os.listdir(HERE) if f.endswith('.hip'))
    common = f'-O3 -fPIC -std=c++17 -D_GLIBCXX_USE_CXX11_ABI={abi} -I{HERE}'
    kflags = f'{common} --offload-arch={ARCH} -munsafe-fp-atomics -Wno-unused-result'
    if VARIANT:
        kflags += ' ' + os.environ.get('MSP_BUILD_DEFINES', '')
    bflags = (f'{common} -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 -DTORCH_EXTENSION_NAME=_C '
              f'-DTORCH_API_INCLUDE_EXTENSION_H -I{ROCM}/include -I{pyinc} -I{pybind11.get_include()} '
              + ' '.join(f'-isystem {p}' for p in tinc) + ' -Wno-deprecated-declarations')
    tlib = os.path.join(tdir, 'lib')
    # Link with the host C++ driver (no --hip-link): the HIP runtime symbols then resolve through
    # libtorch_hip -> torch/lib/libamdhip64.so, i.e. the SAME runtime torch uses (never a 2nd copy).
    ldflags = (f'-shared -fPIC -L{tlib} -Wl,-rpath,{tlib} -Wl,--no-as-needed -lc10 -ltorch -ltorch_cpu '
               f'-ltorch_python -lc10_hip -ltorch_hip')
    out = os.path.join(PKG, '_C.so') if not VARIANT else os.path.join(ROOT, 'build', VARIANT, '_C.so')
    os.makedirs(os.path.dirname(out), exist_ok=True)
    lines = [
        f'hipcc = {hipcc}',
        f'kflags = {kflags}',
        f'bflags = {bflags}',
        f'ldflags = {ldflags}',
        'rule hip\n  command = $hipcc $kflags -c $in -o $out\n  description = HIPCC $in',
        'rule cxx\n  command = $hipcc -x c++ $bflags -c $in -o $out\n  description = CXX $in',
        f'rule link\n  command = {shutil.which("g++") or "g++"} $in $ldflags -o $out\n  description = LINK $out',
    ]
    objs = []
    headers = ' '.join(os.path.join(HERE, h) for h in ('common.h', 'launchers.h'))
    for k in kernels:
        o = os.path.join(BUILD, k.replace('.hip', '.o'))
        lines.append(f'build {o}: hip {os.path.join(HERE, k)} | {headers}')
        objs.append(o)
    bo = os.path.join(BUILD, 'bindings.o')
    lines.append(f'build {bo}: cxx {os.path.join(HERE, "bindings.cpp")} | {headers}')
    objs.append(bo)
    lines.append(f'build {out}: link {" ".join(objs)}')
    os.makedirs(BUILD, exist_ok=True)
    path = os.path.join(BUILD, 'build.ninja')
    with open(path, 'w') as f:
        f.write('\n'.join(lines) + '\n')
    return path, out


def _mtimes(paths):
    return {p: (os.path.getmtime(p) if os.path.exists(p) else None) for p in paths}


def sha256(path):
    import hashlib
    h = hashlib.sha256()
    with open(path, 'rb') as f:
        for chunk in iter(lambda: f.read(1 << 20), b''):
            h.update(chunk)
    return h.hexdigest()


def build(jobs=None, verbose=False, force=None):
    """Incremental ninja build; prints which objects were (re)compiled this call and the sha256 of the
    linked extension, and records both in ``build/BUILD_INFO.json`` (provenance: the same digest is
    printed by ``__graft_entry__.smoke()`` from the .so the GPU process actually loaded).
    ``force`` (or env MSP_FORCE_REBUILD=1): clean first, so every kernel is recompiled."""
    import json
    import time
    path, out = write_ninja(jobs)
    ninja = shutil.which('ninja')
    if ninja is None:
        import ninja as _nj  # pip package ships the binary
        ninja = os.path.join(_nj.BIN_DIR, 'ninja')
    force = os.environ.get('MSP_FORCE_REBUILD') == '1' if force is None else force
    if force:
        subprocess.run([ninja, '-f', path, '-t', 'clean'], check=True, cwd=BUILD, stdout=subprocess.DEVNULL)
    objs = sorted(os.path.join(BUILD, f.replace('.hip', '.o')) for f in os.listdir(HERE) if f.endswith('.hip'))
    objs.append(os.path.join(BUILD, 'bindings.o'))
    before = _mtimes(objs + [out])
    cmd = [ninja, '-f', path]
    if jobs:
        cmd += ['-j', str(jobs)]
    if verbose:
        cmd.append('-v')
    subprocess.run(cmd, check=True, cwd=BUILD)
    after = _mtimes(objs + [out])
    compiled = [os.path.basename(p) for p in objs if after[p] != before[p]]
    info = {'arch': ARCH, 'extension': os.path.relpath(out, ROOT), 'sha256': sha256(out),
            'compiled_this_call': compiled, 'relinked': after[out] != before[out],
            'objects': [os.path.basename(p) for p in objs], 'time': time.strftime('%Y-%m-%d %H:%M:%S')}
    os.makedirs(os.path.join(ROOT, 'build'), exist_ok=True)
    with open(os.path.join(ROOT, 'build', 'BUILD_INFO.json' if not VARIANT else f'BUILD_INFO_{VARIANT}.json'),
              'w') as f:
        json.dump(info, f, indent=1)
    print(f'[build] {ARCH}: compiled {len(compiled)}/{len(objs)} objects this call '
          f'({", ".join(compiled) if compiled else "all up to date"}); '
          f'{"relinked" if info["relinked"] else "unchanged"} {info["extension"]} sha256={info["sha256"][:16]}',
          flush=True)
    return out


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--jobs', type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument('--verbose', action='store_true')
    a = ap.parse_args()
    print(build(a.jobs, a.verbose))
    sys.exit(0)
