"""Loader for the in-tree HIP extension ``medical_segmentation_pytorch_amd._C`` (built by
``csrc/build.py`` / ``__graft_entry__.build()`` for gfx950).

On a GPU box the fused engine REQUIRES the extension: :func:`require` raises instead of silently
falling back to eager PyTorch, so a missing/stale build can never masquerade as the HIP path.
"""
from __future__ import annotations

import os

import torch

_C = None
_ERR = None
try:
    if os.environ.get('MSP_C_SO'):   # a profiling variant of the extension (csrc/build.py MSP_BUILD_VARIANT)
        import importlib.util
        import sys
        _spec = importlib.util.spec_from_file_location('medical_segmentation_pytorch_amd._C', os.environ['MSP_C_SO'])
        _C = importlib.util.module_from_spec(_spec)
        _spec.loader.exec_module(_C)
        sys.modules['medical_segmentation_pytorch_amd._C'] = _C
    else:
        from .. import _C  # noqa: F401
except Exception as e:  # pragma: no cover - depends on build state
    _ERR = e


def tree_sources_sha():
    """sha256 of the csrc/ sources in this tree (``csrc/build.py sources_sha``), or None without them."""
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    path = os.path.join(root, 'csrc', 'build.py')
    if not os.path.isfile(path):
        return None
    import importlib.util
    spec = importlib.util.spec_from_file_location('_msp_csrc_build', path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.sources_sha()


def _check_provenance():
    """Refuse an extension built from other sources than the tree's (a stale prebuilt ``_C.so``): it would
    bench / test kernels the sources do not describe.  env MSP_ALLOW_STALE_EXT=1 skips the check."""
    global _C, _ERR
    if _C is None or os.environ.get('MSP_ALLOW_STALE_EXT') == '1':
        return
    want = tree_sources_sha()
    got = _C.sources_sha() if hasattr(_C, 'sources_sha') else None
    if want is not None and got != want:
        _ERR = RuntimeError(f'stale HIP extension {getattr(_C, "__file__", "?")}: built from sources {got!s:.16}, '
                            f'the tree has {want:.16} -- rebuild with `python csrc/build.py`')
        _C = None


_check_provenance()


def available() -> bool:
    return _C is not None


def stale() -> bool:
    """True when a built extension exists but was refused by the provenance check (sources changed)."""
    return _C is None and isinstance(_ERR, RuntimeError) and 'stale HIP extension' in str(_ERR)


def require():
    if _C is None:
        so = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), '_C.so')
        raise RuntimeError(f'HIP extension not loaded ({so}): {_ERR!r}. Build it with `python csrc/build.py`.')
    return _C


def gpu_ready() -> bool:
    """True when the fused HIP engine can run (extension built AND a ROCm device present)."""
    return available() and torch.cuda.is_available()
