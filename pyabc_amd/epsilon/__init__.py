from .base import Epsilon, NoEpsilon
from .epsilon import (ConstantEpsilon, ListEpsilon, QuantileEpsilon,
                      MedianEpsilon)
from .temperature import (TemperatureBase, ListTemperature, Temperature,
                          TemperatureScheme, AcceptanceRateScheme,
                          ExpDecayFixedIterScheme, ExpDecayFixedRatioScheme,
                          PolynomialDecayFixedIterScheme, DalyScheme,
                          FrielPettittScheme, EssScheme, DeviceRecords,
                          match_acceptance_rate)
