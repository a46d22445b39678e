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
total_nr_simulations, ...) return the reference's pandas shapes.
``sqlite://`` (in memory) keeps everything in HBM / host memory; a file
``sqlite:///path`` is also written in pyABC's schema by the bulk writer of
``sqlite_store`` (libabcstore.so, in the background) and can be resumed with
``ABCSMC.load`` -- including files written by pyABC itself.
"""
import datetime

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

    @classmethod
    def from_host(cls, t, h, model_names):
        """A generation read back from a database file (host only)."""
        g = cls(t, h["epsilon"], h["samples"], None, model_names)
        g.host = h
        g.end_time = h.get("end_time", g.end_time)
        return g

    def host_future(self):
        """Callable returning the host dict; for device populations the
        copies are enqueued now (pinned, async) and waited for on call."""
        pop = self.population
        if pop is None or pop.columns is None:
            return self.to_host
        from .. import gpu
        c = pop.columns
        futs = gpu.HostFuture.group((c.theta, c.weights, c.distances, c.sum_stats))
        names, keys = list(c.param_names), list(c.sum_stat_keys)

        def get():
            th, w, d, ss = (f.get() for f in futs)
            return dict(theta=th, w=w, distance=d, sum_stats=ss, names=names,
                        keys=keys)
        return get

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


def _population_from_host(h):
    """A particle-list Population of a host-only generation (one accepted
    sample per particle, as History stores it)."""
    from ..parameters import Parameter
    from ..population import Particle, Population
    parts = []
    for i in range(len(h["w"])):
        ss = dict(zip(h["keys"], map(float, h["sum_stats"][i]))) \
            if len(h["keys"]) else {}
        parts.append(Particle(
            m=int(h["m"][i]) if "m" in h else 0,
            parameter=Parameter(dict(zip(h["names"], map(float, h["theta"][i])))),
            weight=float(h["w"][i]), accepted_sum_stats=[ss],
            accepted_distances=[float(h["distance"][i])]))
    return Population(parts)


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
        self._store = None
        path = db[len("sqlite:///"):] if db.startswith("sqlite:///") else ""
        if path:
            from .sqlite_store import SQLiteStore
            self._store = SQLiteStore(path)

    def __getstate__(self):
        state = self.__dict__.copy()
        state["_store"] = None          # thread + native handle stay local
        return state

    @property
    def db_file(self):
        return self._store.path if self._store is not None else None

    def load_run(self, abc_id=None):
        """Read a run back from the database file (history.py readers)."""
        from .sqlite_store import read_run
        if self._store is None:
            raise ValueError("load_run needs a sqlite:///path database")
        self._store.flush()
        self.id, gens, meta = read_run(self._store.path, abc_id)
        names = meta.get("model_names", [])
        self._gens = {t: _Gen.from_host(t, h, names) for t, h in gens.items()}
        self._pre_samples = meta["pre_samples"]
        self._meta.update(x_0=meta["x_0"], gt_par=meta["gt_par"],
                          model_names=names)
        return self

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
        if self._store is not None:
            self.id = self._store.new_run(options, distance_function_json_str,
                                          eps_function_json_str,
                                          population_strategy_json_str)
            self._store.store_pre_population(
                self.id, ground_truth_model, observed_summary_statistics,
                ground_truth_parameter, model_names)

    def update_nr_samples(self, t, nr_samples):
        if t == History.PRE_TIME:
            self._pre_samples = int(nr_samples)
        elif t in self._gens:
            self._gens[t].samples = int(nr_samples)
        if self._store is not None:
            self._store.update_nr_samples(self.id, t, nr_samples)

    def append_population(self, t, current_epsilon, population, nr_simulations,
                          model_names):
        g = _Gen(t, current_epsilon, nr_simulations, population, model_names)
        self._gens[t] = g
        if self._store is not None:
            mp = g.model_probabilities()
            if len(mp) > 1:
                raise NotImplementedError(
                    "the file store writes single-model populations")
            m = next(iter(mp)) if mp else 0
            self._store.submit(self.id, t, current_epsilon, nr_simulations,
                               g.host_future(), model_names[m] if model_names
                               else "model", float(mp.get(m, 1.0)), m,
                               self.stores_sum_stats)
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
        if self._store is not None:
            self._store.done(self.id)

    def flush(self):
        """Wait until every population is in the database file."""
        if self._store is not None:
            self._store.flush()

    # -- reading ----------------------------------------------------------
    @property
    def max_t(self):
        return max(self._gens) if self._gens else -1

    @property
    def n_populations(self):
        return len(self._gens)

    @property
    def total_nr_simulations(self):
        # history.py:556-568 sums nr_samples over all populations, the
        # calibration (t = PRE_TIME) included
        return self._pre_samples + sum(g.samples for g in self._gens.values())

    def observed_sum_stat(self):
        return self._meta.get("x_0", {})

    def get_population(self, t=None):
        t = self.max_t if t is None else t
        g = self._gens[t]
        if g.population is not None:
            return g.population
        return _population_from_host(g.to_host())

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
                     particles=1)]       # the ground-truth particle
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
