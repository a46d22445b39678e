"""SQLite file store in pyABC's schema (History with ``sqlite:///path``).

Reference: pyabc/storage/history.py (store_initial_data :374-436,
store_pre_population :438-498, update_nr_samples :500-527, done :604-614,
_save_to_population_db :616-693, the readers get_distribution :268-314,
get_all_populations :345-372, observed_sum_stat :529-554) over the schema of
pyabc/storage/db_model.py:35-127.

Writing: the small run metadata goes through Python's sqlite3 module; every
population goes to ``libabcstore.so`` (include/abcstore.h), a C++ bulk writer
with one prepared statement per table and one transaction per population,
on a background thread.  The ctypes call releases the GIL, and the device ->
host copy is an async pinned copy enqueued when the population is appended,
so the generation loop does not wait for the database.  The resulting file is
the reference's schema, so pyABC's own History can open it; ``read_run``
reads it back (files written by pyABC included) for ``ABCSMC.load``.
"""
import ctypes as C
import datetime
import io
import os
import queue
import sqlite3
import threading

import numpy as np

_HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("ABCSTORE_LIB", os.path.join(_HERE, "libabcstore.so"))

_lib = None
_lock = threading.Lock()


def load():
    """libabcstore.so (host code; built by pyabc_amd.build)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(f"libabcstore.so not found at {LIB_PATH}; "
                                  "build it with `python -m pyabc_amd.build`")
            lib = C.CDLL(LIB_PATH)
            P, I64, I32, D = C.c_void_p, C.c_int64, C.c_int, C.c_double
            CP = C.POINTER(C.c_char_p)
            lib.abc_store_last_error.restype = C.c_char_p
            lib.abc_store_open.argtypes = [C.c_char_p, C.POINTER(C.c_void_p)]
            lib.abc_store_close.argtypes = [P]
            lib.abc_store_exec.argtypes = [P, C.c_char_p]
            lib.abc_store_write_population.argtypes = [
                P, I64, I64, C.c_char_p, I64, D, I64, C.c_char_p, D, I64, I32,
                CP, P, P, P, I32, CP, P, P, I32, C.POINTER(C.c_int64)]
            for f in ("abc_store_open", "abc_store_close", "abc_store_exec",
                      "abc_store_write_population"):
                getattr(lib, f).restype = I32
            _lib = lib
    return _lib


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: {load().abc_store_last_error().decode()}")


def _npy(value):
    """BytesStorage encoding (numpy_bytes_storage.py:6-24)."""
    f = io.BytesIO()
    np.save(f, value, allow_pickle=False)
    return f.getvalue()


_F8_PREFIX = _npy(np.float64(0.0))[:-8]


def _from_npy(blob):
    """numpy_bytes_storage.py:27-59 (no pickles: allow_pickle=False)."""
    if blob[:len(_F8_PREFIX)] == _F8_PREFIX and len(blob) == len(_F8_PREFIX) + 8:
        return float(np.frombuffer(blob, dtype="<f8", offset=len(_F8_PREFIX))[0])
    arr = np.load(io.BytesIO(blob), allow_pickle=False)
    if arr.size == 1:
        for type_ in (int, float, str):
            try:
                if type_(arr) == arr:
                    return type_(arr)
            except (TypeError, ValueError):
                pass
    return arr


def _now():
    return str(datetime.datetime.now())


class SQLiteStore:
    """One database file; populations written in the background."""

    def __init__(self, path):
        self.path = path
        h = C.c_void_p()
        _check(load().abc_store_open(path.encode(), C.byref(h)), "open")
        self._h = h
        load().abc_store_exec(self._h, b"PRAGMA synchronous=OFF")
        self._q = queue.Queue()
        self._err = None
        self._thread = threading.Thread(target=self._worker, daemon=True)
        self._thread.start()

    def _conn(self):
        return sqlite3.connect(self.path, timeout=600)

    # -- metadata (python sqlite3) -----------------------------------------
    def new_run(self, options, distance, epsilon, population_strategy):
        self.flush()
        with self._conn() as con:
            cur = con.execute(
                "INSERT INTO abc_smc (start_time, json_parameters, git_hash, "
                "distance_function, epsilon_function, population_strategy) "
                "VALUES (?, ?, ?, ?, ?, ?)",
                (_now(), str(options), "not a git repository", distance,
                 epsilon, population_strategy))
            return int(cur.lastrowid)

    def store_pre_population(self, abc_id, gt_model, x_0, gt_par, model_names):
        """history.py:438-498: t = -1 with the ground truth and x_0."""
        with self._conn() as con:
            pid = con.execute(
                "INSERT INTO populations (abc_smc_id, t, population_end_time, "
                "nr_samples, epsilon) VALUES (?, -1, ?, 0, ?)",
                (abc_id, _now(), float("inf"))).lastrowid
            name = None if gt_model is None else model_names[gt_model]
            mid = con.execute(
                "INSERT INTO models (population_id, m, name, p_model) "
                "VALUES (?, ?, ?, 1)", (pid, gt_model, name)).lastrowid
            part = con.execute("INSERT INTO particles (model_id, w) VALUES (?, 1)",
                               (mid,)).lastrowid
            con.executemany(
                "INSERT INTO parameters (particle_id, name, value) VALUES (?, ?, ?)",
                [(part, k, float(v)) for k, v in gt_par.items()])
            sid = con.execute("INSERT INTO samples (particle_id, distance) "
                              "VALUES (?, 0)", (part,)).lastrowid
            con.executemany(
                "INSERT INTO summary_statistics (sample_id, name, value) "
                "VALUES (?, ?, ?)",
                [(sid, k, _npy(v)) for k, v in x_0.items()])
            for m, nm in enumerate(model_names):
                if m != gt_model:
                    con.execute("INSERT INTO models (population_id, m, name, "
                                "p_model) VALUES (?, ?, ?, 0)", (pid, m, nm))

    def update_nr_samples(self, abc_id, t, n):
        self.flush()
        with self._conn() as con:
            con.execute("UPDATE populations SET nr_samples = ? WHERE "
                        "abc_smc_id = ? AND t = ?", (int(n), abc_id, int(t)))

    def done(self, abc_id):
        self.flush()
        with self._conn() as con:
            con.execute("UPDATE abc_smc SET end_time = ? WHERE id = ?",
                        (_now(), abc_id))

    # -- populations (libabcstore, background thread) ------------------------
    def submit(self, abc_id, t, eps, n_sim, host_fn, model_name, p_model=1.0,
               m=0, store_sum_stats=True):
        """Queue one population; host_fn() returns the host dict (theta, w,
        distance, sum_stats, names, keys) when the device copy is done."""
        if self._err is not None:
            raise self._err
        self._q.put((abc_id, t, eps, n_sim, host_fn, model_name, p_model, m,
                     store_sum_stats, _now()))

    def _worker(self):
        while True:
            job = self._q.get()
            if job is None:
                self._q.task_done()
                return
            try:
                self._write(*job)
            except Exception as e:          # surfaced by the next submit/flush
                self._err = e
            finally:
                self._q.task_done()

    def _write(self, abc_id, t, eps, n_sim, host_fn, model_name, p_model, m,
               store_sum_stats, end_time):
        h = host_fn()
        theta = np.ascontiguousarray(h["theta"], dtype=np.float64)
        w = np.ascontiguousarray(h["w"], dtype=np.float64)
        dist = np.ascontiguousarray(h["distance"], dtype=np.float64)
        n = w.size
        names, keys = list(h["names"]), list(h["keys"]) if store_sum_stats else []
        ss = (np.ascontiguousarray(h["sum_stats"], dtype=np.float64)
              if keys else np.zeros((n, 0)))
        d, S = len(names), len(keys)
        pn = (C.c_char_p * max(d, 1))(*[s.encode() for s in names])
        sn = (C.c_char_p * max(S, 1))(*[s.encode() for s in keys])
        pid = C.c_int64()
        rc = load().abc_store_write_population(
            self._h, abc_id, int(t), end_time.encode(), int(n_sim), float(eps),
            int(m), str(model_name).encode(), float(p_model), n, d, pn,
            theta.ctypes.data, w.ctypes.data, dist.ctypes.data, S, sn,
            ss.ctypes.data if S else None, _F8_PREFIX, len(_F8_PREFIX),
            C.byref(pid))
        _check(rc, f"write population t={t}")

    def flush(self):
        self._q.join()
        if self._err is not None:
            err, self._err = self._err, None
            raise err

    def close(self):
        if self._h is not None:
            self.flush()
            self._q.put(None)
            self._thread.join()
            load().abc_store_close(self._h)
            self._h = None


def read_run(path, abc_id=None):
    """All populations of one run as host dicts (t -> dict with theta, w,
    distance, sum_stats, names, keys, m, epsilon, samples, end_time,
    model_probabilities) plus the run metadata; reads files written by
    pyABC's History as well as by SQLiteStore."""
    con = sqlite3.connect(path)
    try:
        if abc_id is None:
            abc_id = con.execute("SELECT max(id) FROM abc_smc").fetchone()[0]
        pops = con.execute(
            "SELECT id, t, epsilon, nr_samples, population_end_time FROM "
            "populations WHERE abc_smc_id = ? ORDER BY t", (abc_id,)).fetchall()
        gens, meta = {}, {"x_0": {}, "gt_par": {}, "pre_samples": 0}
        for pid, t, eps, nsamp, end in pops:
            models = con.execute(
                "SELECT id, m, name, p_model FROM models WHERE population_id = ?"
                " ORDER BY m", (pid,)).fetchall()
            if t == -1:
                meta["pre_samples"] = int(nsamp or 0)
                meta["model_names"] = [nm for _, _, nm, _ in models]
                for mid, *_ in models:
                    for k, v in con.execute(
                            "SELECT pa.name, pa.value FROM parameters pa JOIN "
                            "particles p ON pa.particle_id = p.id WHERE "
                            "p.model_id = ?", (mid,)):
                        meta["gt_par"][k] = v
                    for k, v in con.execute(
                            "SELECT ss.name, ss.value FROM summary_statistics ss "
                            "JOIN samples s ON ss.sample_id = s.id JOIN "
                            "particles p ON s.particle_id = p.id WHERE "
                            "p.model_id = ?", (mid,)):
                        meta["x_0"][k] = _from_npy(v)
                continue
            th_all, w_all, d_all, ss_all, m_all = [], [], [], [], []
            names = keys = None
            mp = {}
            for mid, m, _, p_model in models:
                mp[int(m)] = float(p_model)
                parts = con.execute("SELECT id, w FROM particles WHERE model_id "
                                    "= ? ORDER BY id", (mid,)).fetchall()
                if not parts:
                    continue
                ids = np.array([p[0] for p in parts])
                pos = {int(i): j for j, i in enumerate(ids)}
                prm = con.execute(
                    "SELECT pa.particle_id, pa.name, pa.value FROM parameters pa "
                    "JOIN particles p ON pa.particle_id = p.id WHERE p.model_id "
                    "= ?", (mid,)).fetchall()
                nm = sorted({r[1] for r in prm})
                col = {k: j for j, k in enumerate(nm)}
                th = np.full((len(ids), len(nm)), np.nan)
                for partid, k, v in prm:
                    th[pos[partid], col[k]] = v
                smp = con.execute(
                    "SELECT s.id, s.particle_id, s.distance FROM samples s JOIN "
                    "particles p ON s.particle_id = p.id WHERE p.model_id = ? "
                    "ORDER BY s.id", (mid,)).fetchall()
                dist = np.full(len(ids), np.nan)
                first_sample = {}
                for sid, partid, dv in smp:
                    if partid not in first_sample:
                        first_sample[partid] = sid
                        dist[pos[partid]] = dv
                sst = con.execute(
                    "SELECT ss.sample_id, ss.name, ss.value FROM "
                    "summary_statistics ss JOIN samples s ON ss.sample_id = s.id"
                    " JOIN particles p ON s.particle_id = p.id WHERE p.model_id"
                    " = ? ORDER BY ss.id", (mid,)).fetchall()
                ks = []
                for _, k, _ in sst:
                    if k not in ks:
                        ks.append(k)
                kcol = {k: j for j, k in enumerate(ks)}
                srow = {sid: pos[partid] for partid, sid in first_sample.items()}
                ss = np.full((len(ids), len(ks)), np.nan)
                for sid, k, v in sst:
                    if sid in srow:
                        val = _from_npy(v)
                        ss[srow[sid], kcol[k]] = val if np.ndim(val) == 0 else np.nan
                names = nm if names is None else names
                keys = ks if keys is None else keys
                th_all.append(th)
                w_all.append(np.array([p[1] for p in parts], dtype=float))
                d_all.append(dist)
                ss_all.append(ss)
                m_all.append(np.full(len(ids), int(m)))
            gens[int(t)] = dict(
                theta=np.concatenate(th_all) if th_all else np.zeros((0, 0)),
                w=np.concatenate(w_all) if w_all else np.zeros(0),
                distance=np.concatenate(d_all) if d_all else np.zeros(0),
                sum_stats=np.concatenate(ss_all) if ss_all else np.zeros((0, 0)),
                names=names or [], keys=keys or [],
                m=np.concatenate(m_all) if m_all else np.zeros(0, dtype=int),
                model_probabilities=mp, epsilon=float(eps),
                samples=int(nsamp or 0), end_time=end)
        return abc_id, gens, meta
    finally:
        con.close()
