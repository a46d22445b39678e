"""Population size strategies (pyabc/populationstrategy.py:22-129).
AdaptivePopulationSize is outside the hot path."""
import json
import logging

logger = logging.getLogger("Adaptation")


class PopulationStrategy:
    def __init__(self, nr_calibration_particles: int = None,
                 nr_samples_per_parameter: int = 1):
        self.nr_calibration_particles = nr_calibration_particles
        self.nr_samples_per_parameter = nr_samples_per_parameter

    def update(self, transitions, model_weights, t=None):
        pass

    def __call__(self, t: int = None) -> int:
        raise NotImplementedError

    def get_config(self):
        return {"name": self.__class__.__name__,
                "nr_calibration_particles": self.nr_calibration_particles,
                "nr_samples_per_parameter": self.nr_samples_per_parameter}

    def to_json(self):
        return json.dumps(self.get_config())


class ConstantPopulationSize(PopulationStrategy):
    def __init__(self, nr_particles: int, nr_calibration_particles: int = None,
                 nr_samples_per_parameter: int = 1):
        super().__init__(nr_calibration_particles=nr_calibration_particles,
                         nr_samples_per_parameter=nr_samples_per_parameter)
        self.nr_particles = nr_particles

    def __call__(self, t: int = None) -> int:
        if t == -1 and self.nr_calibration_particles is not None:
            return self.nr_calibration_particles
        return self.nr_particles

    def get_config(self):
        config = super().get_config()
        config["nr_particles"] = self.nr_particles
        return config
