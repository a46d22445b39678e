"""Diagnostic: count gave-up proposals per round in a StochasticAcceptor run
with a narrow bounded prior (tests/test_stochastic.py gave-up test)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import pyabc_amd as pa
from pyabc_amd import gpu
np.random.seed(3)
model = pa.LinearGaussianModel(["x"], ["y"], src=[0], sigma=[0.0])
prior = pa.Distribution(x=pa.RV("uniform", 1.2, 0.3))
sampler = pa.BatchedGPUSampler(seed=91, max_attempts=2)
abc = pa.ABCSMC(model, prior, pa.IndependentNormalKernel(var=[0.25]),
                population_size=3000, sampler=sampler,
                transitions=pa.MultivariateNormalTransition(scaling=50),
                eps=pa.Temperature(initial_temperature=8.0), acceptor=pa.StochasticAcceptor())
abc.new("sqlite://", {"y": 2.0})
orig = gpu.mask_gave_up
def spy(dist, att, max_attempts, value=float("nan")):
    a = att.cpu().numpy()
    print("mask: B", a.size, "att hist", np.bincount(a)[:6], "max_att", max_attempts, "value", value, flush=True)
    return orig(dist, att, max_attempts, value)
gpu.mask_gave_up = spy
orig_prop = pa.MultivariateNormalTransition.propose_device
def pspy(self, B, *a, **k):
    print("propose_device B", B, "max_attempts", k.get("max_attempts"), "cov", self.cov, flush=True)
    return orig_prop(self, B, *a, **k)
pa.MultivariateNormalTransition.propose_device = pspy
h = abc.run(max_nr_populations=4)
print("max_t", h.max_t, "temps", abc.eps.temperatures)
