"""Transitions (pyabc/transition/__init__.py): GPU-backed perturbation
kernels behind the reference's Transition API."""
from .base import Transition, DiscreteTransition
from .exceptions import NotEnoughParticles
from .multivariatenormal import (MultivariateNormalTransition,
                                 silverman_rule_of_thumb, scott_rule_of_thumb)
from .local_transition import LocalTransition
from .randomwalk import DiscreteRandomWalkTransition
from .predict_population_size import predict_population_size, CVEstimate

__all__ = ["Transition", "DiscreteTransition", "NotEnoughParticles",
           "MultivariateNormalTransition", "LocalTransition",
           "DiscreteRandomWalkTransition",
           "silverman_rule_of_thumb", "scott_rule_of_thumb",
           "predict_population_size", "CVEstimate"]
