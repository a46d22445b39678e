"""JSON helpers for acceptor / temperature log files
(pyabc/storage/json.py:6-47)."""
import copy
import json

import numpy as np


def save_dict_to_json(dct: dict, file_: str):
    """Write dct (ndarray values as lists); inverse of load_dict_from_json."""
    dct = copy.deepcopy(dct)
    for key, val in dct.items():
        if isinstance(val, np.ndarray):
            dct[key] = list(val)
    with open(file_, 'w') as f:
        json.dump(dct, f)


def load_dict_from_json(file_: str, key_type: type = int):
    """Read a json dict, keys converted to int (json.py:26-47)."""
    with open(file_, 'r') as f:
        _dct = json.load(f)
    return {int(key): val for key, val in _dct.items()}
