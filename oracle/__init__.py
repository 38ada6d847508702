"""CPU oracle for the batched Metropolis-Hastings / CondCov-Gibbs hot path.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this package, and only as the checker (or as the
timed CPU baseline).  The product path (probayes_amd) never imports it.

What it is: a vectorised NumPy/SciPy restatement of the reference's per-chain
step (probayes 0.0.8, /root/reference), one NumPy array lane per chain, that is
bit-identical per chain to the reference's scalar SP.next loop on the same
legacy-MT19937 random streams.  Each function cites the reference file:line it
restates.

Pinning: tests/test_oracle_golden.py checks every workload against the golden
traces in tests/golden/*.npz, which tools/gen_golden.py recorded by running the
reference itself in the build container (numpy 2.2.6, scipy 1.15.3).

Third-party arithmetic the reference delegates: scipy 1.15.3
`norm.logpdf/pdf/ppf/cdf`, `uniform.pdf`, `multivariate_normal.pdf`,
`special.ndtri`; numpy 2.2.6 legacy `RandomState` (MT19937 + polar gauss) and
its pairwise `np.sum`.  The oracle calls the same functions the reference calls.
"""
from oracle.streams import legacy_streams, stream_width  # noqa: F401
from oracle.mh import run_mh  # noqa: F401
from oracle.gibbs import run_gibbs, condcov_tables  # noqa: F401
from oracle.workloads import WORKLOADS, load_golden, golden_spec  # noqa: F401
