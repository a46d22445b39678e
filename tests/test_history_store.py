"""History file store in pyABC's SQLite schema.

Pinning (tests/golden/make_golden.py --history, importing pyABC 0.10.5):
* ``ref_history.db`` is a 2-generation run stored by pyABC's own History;
  ``read_run`` / ``ABCSMC.load`` must read back exactly what pyABC's
  readers returned (history.npz: theta, w, distances, population table);
* a file written by ``libabcstore`` (the bulk writer) was read with pyABC's
  History when the fixture was made: the values it returned equal the
  arrays written (ours_ref_* == ours_*), so the format is pyABC-readable.
CPU only: the writer and reader are host code.
"""
import os
import shutil
import sqlite3

import numpy as np
import pytest

from conftest import GOLDEN

G = np.load(os.path.join(GOLDEN, "history.npz"))


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from pyabc_amd import build
    build.build_store(verbose=False)


def _ref_copy(tmp_path):
    p = str(tmp_path / "ref.db")
    shutil.copy(os.path.join(GOLDEN, "ref_history.db"), p)
    return p


def test_reference_written_file_reads_back(tmp_path):
    from pyabc_amd.storage.sqlite_store import read_run
    abc_id, gens, meta = read_run(_ref_copy(tmp_path), 1)
    assert meta["x_0"] == {"y": 2.0, "z": 4.0} and meta["gt_par"] == {"x": 1.5}
    for t in (0, 1):
        h = gens[t]
        np.testing.assert_array_equal(h["theta"][:, 0], G[f"theta_{t}"])
        np.testing.assert_allclose(h["w"] / h["w"].sum(), G[f"w_{t}"],
                                   rtol=1e-15)
        np.testing.assert_array_equal(h["distance"], G[f"dist_{t}"])
        assert h["keys"] == ["y", "z"]
        np.testing.assert_allclose(h["sum_stats"][:, 1], 2 * h["theta"][:, 0],
                                   rtol=1e-15)


def test_abcsmc_load_from_reference_file(tmp_path):
    import pyabc_amd as pa
    p = _ref_copy(tmp_path)
    abc = pa.ABCSMC(lambda par: {"y": par["x"]},
                    pa.Distribution(x=pa.RV("norm", 0, 1)))
    h = abc.load("sqlite:///" + p, 1)
    assert h.max_t == 1 and abc.x_0 == {"y": 2.0, "z": 4.0}
    for t in (0, 1):
        df, w = h.get_distribution(0, t)
        np.testing.assert_array_equal(df["x"].values, G[f"theta_{t}"])
        np.testing.assert_allclose(w, G[f"w_{t}"], rtol=1e-15)
    pops = h.get_all_populations()
    np.testing.assert_array_equal(
        pops[["t", "samples", "epsilon", "particles"]].values.astype(float),
        G["pops"])
    pop = h.get_population(1)
    assert len(pop) == 40


def test_bulk_writer_is_reference_readable():
    """Values pyABC's History read from a libabcstore file (fixture time)."""
    np.testing.assert_array_equal(G["ours_ref_theta"], G["ours_theta"])
    np.testing.assert_allclose(G["ours_ref_w"], G["ours_w"] / G["ours_w"].sum(),
                               rtol=1e-15)
    np.testing.assert_array_equal(G["ours_ref_dist"], G["ours_dist"])
    np.testing.assert_array_equal(G["ours_ref_ss"], G["ours_ss"])
    np.testing.assert_array_equal(G["ours_ref_x0"], [1.0, 2.0])
    np.testing.assert_array_equal(G["ours_ref_pops"],
                                  [[-1, 77, np.inf, 1], [0, 123, 0.7, 50]])
    assert int(G["ours_ref_nsim"]) == 77 + 123


def test_schema_matches_reference(tmp_path):
    from pyabc_amd.storage.sqlite_store import SQLiteStore

    def cols(path):
        con = sqlite3.connect(path)
        tabs = [r[0] for r in con.execute(
            "SELECT name FROM sqlite_master WHERE type='table' ORDER BY name")]
        out = {t: [r[1:3] for r in con.execute(f"PRAGMA table_info({t})")]
               for t in tabs}
        con.close()
        return out
    p = str(tmp_path / "ours.db")
    SQLiteStore(p).close()
    assert cols(p) == cols(_ref_copy(tmp_path))


def test_history_write_read_round_trip(tmp_path):
    """History(sqlite:///file) with a particle-list population: written in
    the background by libabcstore, read back by read_run and ABCSMC.load."""
    import pyabc_amd as pa
    from pyabc_amd.storage.sqlite_store import read_run
    p = str(tmp_path / "rt.db")
    h = pa.History("sqlite:///" + p)
    h.store_initial_data(None, {}, {"s0": 1.0, "s1": np.array([1.0, 2.0])},
                         {}, ["m0"], "{}", "{}", "{}")
    rng = np.random.default_rng(1)
    th, w, d, ss = (rng.normal(size=(30, 2)), rng.random(30), rng.random(30),
                    rng.normal(size=(30, 2)))
    w = w / w.sum()
    for t in range(3):
        parts = [pa.Particle(m=0, parameter=pa.Parameter(a=th[i, 0] + t, b=th[i, 1]),
                             weight=w[i],
                             accepted_sum_stats=[{"s0": ss[i, 0], "s1": ss[i, 1]}],
                             accepted_distances=[d[i]]) for i in range(30)]
        h.append_population(t, 1.0 / (t + 1), pa.Population(parts), 100 + t,
                            ["m0"])
    h.update_nr_samples(pa.History.PRE_TIME, 55)
    h.done()
    abc_id, gens, meta = read_run(p)
    assert abc_id == h.id and sorted(gens) == [0, 1, 2]
    assert np.array_equal(meta["x_0"]["s1"], [1.0, 2.0])
    for t in range(3):
        g = gens[t]
        np.testing.assert_array_equal(g["theta"], th + [t, 0])
        np.testing.assert_allclose(g["w"], w, rtol=1e-15)
        np.testing.assert_array_equal(g["distance"], d)
        np.testing.assert_array_equal(g["sum_stats"], ss)
        assert g["samples"] == 100 + t and g["epsilon"] == 1.0 / (t + 1)
    assert meta["pre_samples"] == 55
    h2 = pa.History("sqlite:///" + p).load_run()
    assert h2.total_nr_simulations == 55 + 100 + 101 + 102


@pytest.mark.gpu
def test_batched_run_file_store_and_resume(tmp_path):
    """A batched GPU run writes every device population to the file in the
    background; the file reads back equal to the in-HBM history, and
    ABCSMC.load resumes the run from it."""
    import pyabc_amd as pa
    p = str(tmp_path / "run.db")
    model = pa.LinearGaussianModel(["x"], ["y"], src=[0], sigma=[0.5])
    prior = pa.Distribution(x=pa.RV("norm", 0, 1))

    def make():
        return pa.ABCSMC(model, prior, pa.PNormDistance(), population_size=2000,
                         sampler=pa.BatchedGPUSampler(seed=11))
    abc = make()
    abc.new("sqlite:///" + p, {"y": 2.0})
    h = abc.run(max_nr_populations=3)
    h2 = pa.History("sqlite:///" + p).load_run(h.id)
    assert h2.max_t == h.max_t == 2
    for t in range(3):
        df, w = h.get_distribution(0, t)
        df2, w2 = h2.get_distribution(0, t)
        np.testing.assert_array_equal(df["x"].values, df2["x"].values)
        np.testing.assert_allclose(w, w2, rtol=1e-15)
    assert h2.total_nr_simulations == h.total_nr_simulations
    abc2 = make()
    abc2.load("sqlite:///" + p, h.id)
    h3 = abc2.run(max_nr_populations=1)
    assert h3.max_t == 3
    df, w = h3.get_distribution(0, 3)
    assert abs(float((df["x"].values * w).sum()) - 1.6) < 0.1
