# Adapted from pyABC (https://github.com/ICB-DCM/pyABC), BSD-3-Clause,
# Copyright 2017 the pyABC developers -- see NOTICE at the repository root.
"""Model parameters (pyabc/parameters.py:9-93), same behaviour."""


class ParameterStructure(dict):
    @staticmethod
    def flatten_dict(dict_: dict):
        new_dict = {}
        for key, value in dict_.items():
            if isinstance(value, dict):
                flattened = ParameterStructure.flatten_dict(value)
                for key_flat, value_flat in flattened.items():
                    new_dict.update({str(key) + "." + key_flat: value_flat})
            else:
                new_dict.update({key: value})
        return new_dict

    def __init__(self, *args, **kwargs):
        if len(args) > 0 and len(kwargs) > 0:
            raise Exception("Only keyword or dictionary allowed")
        if len(args) > 0:
            flattened = ParameterStructure.flatten_dict(args[0])
        elif len(kwargs) > 0:
            flattened = ParameterStructure.flatten_dict(kwargs)
        else:
            flattened = {}
        super().__init__(flattened)


class Parameter(ParameterStructure):
    """Dictionary of parameter values with key-wise + and -."""

    def __add__(self, other):
        return Parameter(**{key: self[key] + other[key] for key in self})

    def __sub__(self, other):
        return Parameter(**{key: self[key] - other[key] for key in self})

    def __repr__(self):
        return "<Parameter " + super().__repr__()[1:-1] + ">"

    def __getattr__(self, item):
        try:
            return self[item]
        except KeyError:
            raise AttributeError(item)

    def __getstate__(self):
        return dict(self)

    def __setstate__(self, state):
        self.update(state)

    def copy(self):
        return Parameter(**self)
