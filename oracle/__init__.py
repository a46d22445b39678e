"""CPU oracle: a float64 numpy restatement of pyABC 0.10.5's hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in ``pyabc_amd`` imports this package; only
``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` use it, and only as the checker / the timed CPU reference.  The
product path runs the HIP kernels in ``libabcgpu.so`` and fails loudly when
that library is missing.

Every function cites the reference file:line it restates
(``/root/reference/pyabc/...``).  The restatement is pinned two ways
(DESIGN.md "Parity"):

* against the reference's own known-answer tests (re-stated in
  ``tests/test_oracle_golden.py``), and
* against golden vectors produced by importing the reference in the build
  container (``tests/golden/make_golden.py`` -> ``tests/golden/*.npz``).
"""
from .transition import (smart_cov, silverman_rule_of_thumb, mvn_fit,
                         mvn_logpdf, mvn_pdf, local_k, local_fit,
                         local_logpdf, local_pdf, psd_decompose)
from .distance import (pnorm, standard_deviation, median_absolute_deviation,
                       adaptive_weights)
from .epsilon import weighted_quantile, quantile_epsilon
from .philox import philox4x32_10, uniform01, normal_pairs
from .cv import (bootstrap_variation, mvn_bootstrap_densities,
                 mvn_calc_cv)
from .generation import (effective_sample_size, normalize_weights,
                         importance_weights)
