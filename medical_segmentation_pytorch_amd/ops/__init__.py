"""Fused MI355X operators (autograd Functions over the HIP kernels in ``csrc/``) plus pure-PyTorch
reference implementations used on CPU and in the numerics tests."""
from ._ext import available, gpu_ready, require
from .fm import cpad

__all__ = ['available', 'gpu_ready', 'require', 'cpad']
