"""Distances (pyabc/distance/__init__.py): p-norm distances on the GPU."""
from .base import (Distance, NoDistance, IdentityFakeDistance,
                   AcceptAllDistance, SimpleFunctionDistance, to_distance)
from .distance import PNormDistance, AdaptivePNormDistance, SumStatMatrix
from .scale import (median_absolute_deviation, mean_absolute_deviation,
                    standard_deviation, bias, root_mean_square_deviation,
                    median_absolute_deviation_to_observation,
                    mean_absolute_deviation_to_observation,
                    combined_median_absolute_deviation,
                    combined_mean_absolute_deviation,
                    standard_deviation_to_observation, span, mean, median)
from .kernel import (SCALE_LIN, SCALE_LOG, SCALES, StochasticKernel,
                     SimpleFunctionKernel, NormalKernel,
                     IndependentNormalKernel, IndependentLaplaceKernel,
                     BinomialKernel, PoissonKernel, NegativeBinomialKernel,
                     binomial_pdf_max)
