"""Behaviour of the plugin API at the drop-in boundary, restating the
reference's own tests (pyABC 0.10.5, test/base):

  test_transition.py:15-160  return types, column-order invariance, the
                             0 / 1 / 2 / 20-particle fits, score
  test_stop_sampling.py      min_acceptance_rate, check_max_eval
  test_resume_run.py         load a run from its database and continue
  test_samplers.py:66-72, 235-243   SamplerMeta count assertion

for both transitions on the GPU and for the per-particle and batched
samplers.  These pin behaviour (types, errors, stopping rules), not values.
"""
import numpy as np
import pandas as pd
import pytest
import scipy.stats as st

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(params=["LocalTransition", "MultivariateNormalTransition"])
def transition(request):
    import pyabc_amd as pa
    return getattr(pa, request.param)()


def data(n, cols=("a", "b")):
    df = pd.DataFrame({c: np.random.rand(n) for c in cols})
    return df, np.ones(len(df)) / max(len(df), 1)


def test_rvs_return_type(transition):
    df, w = data(20)
    transition.fit(df, w)
    sample = transition.rvs()
    assert isinstance(sample, pd.Series)
    assert (sample.index == pd.Index(["a", "b"])).all()
    many = transition.rvs(7)
    assert isinstance(many, pd.DataFrame) and many.shape == (7, 2)
    assert list(many.columns) == ["a", "b"]


def test_pdf_return_types(transition):
    df, w = data(20)
    transition.fit(df, w)
    single = transition.pdf(df.iloc[0])
    multiple = transition.pdf(df)
    assert isinstance(single, float)
    assert multiple.shape == (20,)
    np.testing.assert_allclose(multiple[0], single, rtol=1e-12)


def test_argument_order(transition):
    """test_transition.py:142-154: the pdf sorts the parameters itself."""
    df, w = data(20)
    transition.fit(df, w)
    test = df.iloc[0]
    reversed_ = test[::-1]
    assert (np.array(test) != np.array(reversed_)).all()
    assert transition.pdf(test) == transition.pdf(reversed_)


def test_0_particles_fit(transition):
    import pyabc_amd as pa
    df, w = data(0)
    with pytest.raises(pa.NotEnoughParticles):
        transition.fit(df, w)


@pytest.mark.parametrize("n", [1, 2, 20])
def test_few_particles_fit_and_sample(transition, n):
    df, w = data(n)
    transition.fit(df, w)
    transition.required_nr_samples(.1)
    assert np.isfinite(transition.pdf(df)).all()
    assert transition.rvs().shape == (2,)


def test_single_parameter(transition):
    df, w = data(20, cols=("a",))
    transition.fit(df, w)
    transition.required_nr_samples(.1)
    assert transition.rvs().index.tolist() == ["a"]


def test_fit_normalises_weights_in_place(transition):
    """transitionmeta.py:8-21: w / w.sum() written back into the caller's
    array."""
    df, _ = data(20)
    w = np.arange(1.0, 21.0)
    transition.fit(df, w)
    np.testing.assert_allclose(w.sum(), 1.0, rtol=1e-14)


def test_score(transition):
    df, w = data(20)
    transition.fit(df, w)
    assert np.isfinite(transition.score(df, w))


# ---- stopping rules (test_stop_sampling.py) ---------------------------------

def _stop_model(x):
    return {"par": x["par"] + np.random.randn()}


def _stop_dist(x, y):
    return abs(x["par"] - y["par"])


def test_stop_acceptance_rate_too_low():
    import pyabc_amd as pa
    np.random.seed(1)
    abc = pa.ABCSMC(_stop_model, pa.Distribution(par=st.uniform(0, 10)),
                    _stop_dist, 10)
    abc.new("sqlite://", {"par": .5})
    history = abc.run(-1, 8, min_acceptance_rate=0.2)
    df = history.get_all_populations()
    df["acceptance_rate"] = df["particles"] / df["samples"]
    assert df["acceptance_rate"].iloc[-1] < 0.2
    assert df["acceptance_rate"].iloc[-2] >= 0.2 or df["t"].iloc[-2] == -1


def test_stop_early_check_max_eval():
    import pyabc_amd as pa
    np.random.seed(2)
    abc = pa.ABCSMC(_stop_model, pa.Distribution(par=st.uniform(0, 10)),
                    _stop_dist, 10, sampler=pa.SingleCoreSampler(check_max_eval=True))
    abc.new("sqlite://", {"par": .5})
    history = abc.run(max_nr_populations=8, min_acceptance_rate=0.2)
    df = history.get_all_populations()
    assert (df["particles"] / df["samples"]).iloc[-1] >= 0.2


def test_stop_early_batched_check_max_eval():
    """The batched sampler stops a generation at max_eval when asked; the
    run then ends without appending it (smc.py:905-911)."""
    import pyabc_amd as pa
    model = pa.LinearGaussianModel(["x"], ["y"], src=[0], sigma=[0.5])
    abc = pa.ABCSMC(model, pa.Distribution(x=pa.RV("norm", 0, 1)),
                    pa.PNormDistance(), population_size=2000,
                    sampler=pa.BatchedGPUSampler(seed=4, check_max_eval=True))
    abc.new("sqlite://", {"y": 2.0})
    history = abc.run(max_nr_populations=10, min_acceptance_rate=0.3)
    df = history.get_all_populations()
    assert (df["particles"] / df["samples"]).iloc[1:].min() >= 0.3
    assert history.max_t < 9


# ---- resume (test_resume_run.py) ---------------------------------------------

@pytest.mark.parametrize("gt_model", [0, None])
def test_resume(tmp_path, gt_model):
    import pyabc_amd as pa

    def model(parameter):
        return {"data": parameter["mean"] + np.random.randn()}
    prior = pa.Distribution(mean=pa.RV("uniform", 0, 5))

    def distance(x, y):
        return abs(x["data"] - y["data"])
    db = "sqlite:///" + str(tmp_path / "resume.db")
    abc = pa.ABCSMC(model, prior, distance, population_size=10)
    history = abc.new(db, {"data": 2.5}, gt_model=gt_model)
    run_id = history.id
    hist_new = abc.run(minimum_epsilon=0, max_nr_populations=1)
    assert hist_new.n_populations == 1
    abc_continued = pa.ABCSMC(model, prior, distance)
    abc_continued.load(db, run_id)
    hist_contd = abc_continued.run(minimum_epsilon=0, max_nr_populations=1)
    assert hist_contd.n_populations == 2
    assert pa.History(db).load_run(run_id).n_populations == 2


# ---- SamplerMeta (test_samplers.py:66-72, 235-243) ---------------------------

def test_wrong_output_sampler():
    import pyabc_amd as pa

    class WrongOutputSampler(pa.SingleCoreSampler):
        def sample_until_n_accepted(self, n, simulate_one, max_eval=np.inf,
                                    all_accepted=False, show_progress=False):
            return super().sample_until_n_accepted(
                n + 1, simulate_one, max_eval, all_accepted=False,
                show_progress=show_progress)

    def simulate_one():
        return pa.Particle(m=0, parameter={}, weight=0,
                           accepted_sum_stats=[], accepted_distances=[],
                           accepted=True)
    with pytest.raises(AssertionError):
        WrongOutputSampler().sample_until_n_accepted(5, simulate_one)


# ---- two competing models (test_samplers.py:128-209) ----------------------------

@pytest.mark.parametrize("n_sim", [1, 2])
def test_two_competing_gaussians_multiple_population(n_sim):
    """Model selection through the per-particle sampler (PNormDistance in
    place of the reference's PercentileDistance): the run completes, model
    probabilities are numbers, calibration used exactly nr_particles
    evaluations."""
    import pyabc_amd as pa
    np.random.seed(3)
    sigma = .5

    def model(args):
        return {"y": st.norm(args['x'], sigma).rvs()}
    models = list(map(pa.SimpleModel, [model, model]))
    priors = [pa.Distribution(x=pa.RV("norm", 0, sigma)),
              pa.Distribution(x=pa.RV("norm", 1, sigma))]
    pop_size = pa.ConstantPopulationSize(23, nr_samples_per_parameter=n_sim)
    abc = pa.ABCSMC(models, priors, pa.PNormDistance(), pop_size,
                    eps=pa.MedianEpsilon())
    abc.new("sqlite://", {"y": 1})
    history = abc.run(.05, max_nr_populations=2)
    assert history.max_t == 1
    mp = history.get_model_probabilities(history.max_t)
    assert abs(float(mp.p.sum()) - 1.0) < 1e-12
    pops = history.get_all_populations()
    pre_evals = pops[pops['t'] == pa.History.PRE_TIME]['samples'].values
    assert pre_evals == pop_size.nr_particles
