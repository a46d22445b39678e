"""Samplers (pyabc/sampler/__init__.py).  ``BatchedGPUSampler`` is the
MI355X generation engine; ``SingleCoreSampler`` keeps the reference's
per-candidate loop (its plugin calls still run on the GPU)."""
from .base import Sample, SampleFactory, Sampler
from .singlecore import SingleCoreSampler
from .batched import BatchedGPUSampler, ColumnarSample

__all__ = ["Sample", "SampleFactory", "Sampler", "SingleCoreSampler",
           "BatchedGPUSampler", "ColumnarSample"]
