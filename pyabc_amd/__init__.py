"""pyabc_amd: pyABC 0.10.5's ABC-SMC generation engine, MI355X-native.

The public names mirror ``pyabc`` so scripts switch by changing the import.
The hot path (transition fit/rvs/pdf, distances, epsilon quantile, batched
sampling) runs as hand-written HIP kernels in ``libabcgpu.so`` (C ABI,
include/abcgpu.h) loaded through ctypes; see DESIGN.md.
"""
import logging
import os

from .parameters import Parameter
from .random_variables import (Distribution, RV, RVBase, RVDecorator,
                               LowerBoundDecorator)
from .distance import (Distance, NoDistance, IdentityFakeDistance,
                       AcceptAllDistance, SimpleFunctionDistance,
                       PNormDistance, AdaptivePNormDistance, to_distance,
                       StochasticKernel, SimpleFunctionKernel, NormalKernel,
                       IndependentNormalKernel, IndependentLaplaceKernel,
                       BinomialKernel, PoissonKernel, NegativeBinomialKernel)
from .epsilon import (Epsilon, NoEpsilon, ConstantEpsilon, QuantileEpsilon,
                      MedianEpsilon, ListEpsilon, TemperatureBase,
                      ListTemperature, Temperature, TemperatureScheme,
                      AcceptanceRateScheme, ExpDecayFixedIterScheme,
                      ExpDecayFixedRatioScheme,
                      PolynomialDecayFixedIterScheme, DalyScheme,
                      FrielPettittScheme, EssScheme)
from .sampler import (Sampler, Sample, SingleCoreSampler, BatchedGPUSampler)
from .smc import ABCSMC, GenerationSpec, ModelPerturbationKernel
from .storage import History, create_sqlite_db_id
from .acceptor import (Acceptor, SimpleFunctionAcceptor, UniformAcceptor,
                       StochasticAcceptor, pdf_norm_from_kernel,
                       pdf_norm_max_found, ScaledPDFNorm)
from . import distance, epsilon, acceptor, storage
from .model import (Model, SimpleModel, ModelResult, IntegratedModel,
                    VectorizedModel, LinearGaussianModel)
from .transition import (Transition, MultivariateNormalTransition,
                         LocalTransition, DiscreteRandomWalkTransition,
                         NotEnoughParticles)
from .population import Particle, Population
from .populationstrategy import (ConstantPopulationSize, PopulationStrategy,
                                 AdaptivePopulationSize, ListPopulationSize)
from .weighted_statistics import (weighted_quantile, weighted_median,
                                  weighted_mean, weighted_std,
                                  effective_sample_size)

__version__ = "0.1.0"

try:
    loglevel = os.environ['ABC_LOG_LEVEL'].upper()
except KeyError:
    loglevel = 'INFO'
logging.basicConfig(level=loglevel)
