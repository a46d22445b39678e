"""History: the per-generation store ABCSMC reads and writes.

Reference: pyabc/storage/history.py:104-1229 (SQLAlchemy ORM, one row per
particle / parameter / sum stat; SURVEY.md §8f row 1 ranks a faster writer as
the next component after the hot path).  This store keeps every generation
columnar and HBM-resident: populations stay on the GPU as device tensors (no
host round trip inside the generation loop) until the resident history
exceeds ``History.DEVICE_BUDGET``; older ones then move to host numpy.  Host
copies are made on first query only.
The query methods ABCSMC and users need (get_distribution,
get_model_probabilities, get_population, get_all_populations, max_t,
total_nr_simulations, ...) return the reference's pandas shapes.  The
``db`` string is kept for API compatibility; an optional ``sqlite:///path``
is written with a bulk (executemany) writer in ``done()``.
"""
import datetime
import json
import sqlite3

import numpy as np
import pandas as pd


def create_sqlite_db_id(dir_=None, file_="pyabc_test.db"):
    import os
    import tempfile
    if dir_ is None:
        dir_ = tempfile.gettempdir()
    return "sqlite:///" + os.path.join(dir_, file_)


class _Gen:
    def __init__(self, t, eps, n_sim, population, model_names):
        self.t = t
        self.epsilon = float(eps)
        self.samples = int(n_sim)
        self.population = population
        self.model_names = model_names
        self.end_time = datetime.datetime.now()
        self.host = None

    def to_host(self):
        if self.host is not None:
            return self.host
        pop = self.population
        if pop.columns is not None:
            c = pop.columns
            self.host = dict(theta=c.theta.cpu().numpy(), w=c.weights.cpu().numpy(),
                             distance=c.distances.cpu().numpy(),
                             sum_stats=c.sum_stats.cpu().numpy(),
                             names=list(c.param_names),
                             keys=list(c.sum_stat_keys),
                             m=np.zeros(len(c), dtype=int))
        else:
            lst = pop.get_list()
            names = sorted(lst[0].parameter.keys()) if lst else []
            mp = pop.get_model_probabilities()
            keys = list(lst[0].accepted_sum_stats[0].keys()) if lst else []
            self.host = dict(
                theta=np.array([[p.parameter[k] for k in names] for p in lst]),
                w=np.array([p.weight for p in lst]),
                distance=np.array([p.accepted_distances[0] for p in lst]),
                sum_stats=np.array([[p.accepted_sum_stats[0].get(k, np.nan)
                                     for k in keys] for p in lst]),
                names=names, keys=keys, m=np.array([p.m for p in lst]),
                model_probabilities=mp)
        return self.host

    def model_probabilities(self):
        pop = self.population
        if self.host is None and pop is not None and pop.columns is not None:
            return {pop.columns.m: 1.0}      # single-model columnar population
        return self.to_host().get("model_probabilities") or {0: 1.0}

    def device_bytes(self):
        pop = self.population
        if pop is None or pop.columns is None:
            return 0
        c = pop.columns
        return sum(t.numel() * t.element_size()
                   for t in (c.theta, c.weights, c.distances, c.sum_stats)
                   if t is not None)

    def offload(self):
        """Drop the device copy once the generation is no longer needed."""
        self.to_host()
        self.population = None


class History:
    PRE_TIME = -1

    # generations stay in HBM (288 GB per MI355X) until the device-resident
    # history exceeds this many bytes; then the oldest are moved to the host
    DEVICE_BUDGET = 16 << 30

    def __init__(self, db: str = "sqlite://", stores_sum_stats: bool = True):
        self.db = db
        self.id = 1
        self.stores_sum_stats = stores_sum_stats
        self._gens = {}
        self._pre_samples = 0
        self.start_time = None
        self.end_time = None
        self._meta = {}

    # -- writing ----------------------------------------------------------
    def store_initial_data(self, ground_truth_model, options, observed_summary_statistics,
                           ground_truth_parameter, model_names,
                           distance_function_json_str, eps_function_json_str,
                           population_strategy_json_str):
        self._meta = dict(gt_model=ground_truth_model, options=options,
                          x_0=observed_summary_statistics,
                          gt_par=ground_truth_parameter,
                          model_names=model_names,
                          distance=distance_function_json_str,
                          epsilon=eps_function_json_str,
                          population_strategy=population_strategy_json_str)

    def update_nr_samples(self, t, nr_samples):
        if t == History.PRE_TIME:
            self._pre_samples = int(nr_samples)

    def append_population(self, t, current_epsilon, population, nr_simulations,
                          model_names):
        self._gens[t] = _Gen(t, current_epsilon, nr_simulations, population,
                             model_names)
        # keep generations device-resident (no host round trip inside the
        # generation loop); offload the oldest beyond the HBM budget
        resident = sorted(tt for tt, g in self._gens.items()
                          if g.population is not None)
        used = sum(self._gens[tt].device_bytes() for tt in resident)
        for tt in resident[:-2]:
            if used <= self.DEVICE_BUDGET:
                break
            used -= self._gens[tt].device_bytes()
            self._gens[tt].offload()

    def done(self):
        self.end_time = datetime.datetime.now()
        if self.db.startswith("sqlite:///"):
            self._write_sqlite(self.db[len("sqlite:///"):])

    def _write_sqlite(self, path):
        con = sqlite3.connect(path)
        cur = con.cursor()
        cur.execute("CREATE TABLE IF NOT EXISTS populations (abc_id INTEGER, t "
                    "INTEGER, epsilon REAL, nr_samples INTEGER)")
        cur.execute("CREATE TABLE IF NOT EXISTS particles (abc_id INTEGER, t "
                    "INTEGER, m INTEGER, w REAL, distance REAL, params TEXT)")
        for t, g in sorted(self._gens.items()):
            cur.execute("INSERT INTO populations VALUES (?,?,?,?)",
                        (self.id, t, g.epsilon, g.samples))
            h = g.to_host()
            rows = [(self.id, t, int(h["m"][i]), float(h["w"][i]),
                     float(h["distance"][i]),
                     json.dumps(dict(zip(h["names"], map(float, h["theta"][i])))))
                    for i in range(len(h["w"]))]
            cur.executemany("INSERT INTO particles VALUES (?,?,?,?,?,?)", rows)
        con.commit()
        con.close()

    # -- reading ----------------------------------------------------------
    @property
    def max_t(self):
        return max(self._gens) if self._gens else -1

    @property
    def n_populations(self):
        return len(self._gens)

    @property
    def total_nr_simulations(self):
        return sum(g.samples for g in self._gens.values())

    def observed_sum_stat(self):
        return self._meta.get("x_0", {})

    def get_population(self, t=None):
        t = self.max_t if t is None else t
        g = self._gens[t]
        if g.population is not None:
            return g.population
        raise KeyError(f"population {t} is no longer device resident")

    def get_population_device(self, t=None):
        t = self.max_t if t is None else t
        g = self._gens.get(t)
        if g is None or g.population is None:
            return None
        return g.population.columns

    def get_distribution(self, m=0, t=None):
        """(DataFrame of parameters [sorted names], normalised weights)
        (history.py:268-314)."""
        t = self.max_t if t is None else t
        h = self._gens[t].to_host()
        sel = h["m"] == m
        df = pd.DataFrame(h["theta"][sel], columns=h["names"])
        w = h["w"][sel]
        w = w / w.sum() if w.size else w
        return df, w

    def get_model_probabilities(self, t=None):
        t = self.max_t if t is None else t
        if t not in self._gens:
            return pd.DataFrame({"p": []})
        mp = self._gens[t].model_probabilities()
        return pd.DataFrame({"p": list(mp.values())}, index=list(mp.keys()))

    def model_probabilities_dict(self, t=None):
        """{m: p_m} without building a DataFrame (hot loop)."""
        t = self.max_t if t is None else t
        if t not in self._gens:
            return {}
        return dict(self._gens[t].model_probabilities())

    def alive_models(self, t=None):
        return [m for m, pm in self.model_probabilities_dict(t).items() if pm > 0]

    def nr_of_models_alive(self, t=None):
        return len(self.alive_models(t))

    def get_all_populations(self):
        rows = [dict(t=History.PRE_TIME, population_end_time=self.start_time,
                     samples=self._pre_samples, epsilon=np.inf,
                     particles=0)]
        for t, g in sorted(self._gens.items()):
            rows.append(dict(t=t, population_end_time=g.end_time,
                             samples=g.samples, epsilon=g.epsilon,
                             particles=len(g.to_host()["w"])))
        return pd.DataFrame(rows)

    def get_weighted_distances(self, t=None):
        t = self.max_t if t is None else t
        h = self._gens[t].to_host()
        return pd.DataFrame({"distance": h["distance"], "w": h["w"]})

    def get_weighted_sum_stats(self, t=None):
        t = self.max_t if t is None else t
        h = self._gens[t].to_host()
        return list(h["w"]), [dict(zip(h["keys"], row)) for row in h["sum_stats"]]
