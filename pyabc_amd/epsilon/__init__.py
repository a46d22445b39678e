from .base import Epsilon, NoEpsilon
from .epsilon import (ConstantEpsilon, ListEpsilon, QuantileEpsilon,
                      MedianEpsilon)
