"""probayes_amd -- an MI355X-native batched Metropolis-Hastings engine with
the SD/SP stochastic-process API of probayes (Bhumbra/probayes 0.0.8).

The hot path (proposal, joint log-density, accept/reject, CondCov Gibbs) runs
in hand-written gfx950 HIP kernels in libpbhip.so, bound through a ctypes
C-ABI (include/pbhip.h).  There is no CPU fallback.
"""
__version__ = '0.1.0'

from probayes_amd.spec import make_spec, normalize_spec  # noqa: F401
from probayes_amd.engine import Engine  # noqa: F401
from probayes_amd.rv import RV, RF  # noqa: F401,E402
from probayes_amd.sp import SP  # noqa: F401,E402
from probayes_amd.pd import PD  # noqa: F401,E402
from probayes_amd.lower import NotLowerable  # noqa: F401,E402
from probayes_amd import models  # noqa: F401,E402
from probayes_amd import likelihoods  # noqa: F401,E402
from probayes_amd.likelihoods import bool_perm_freq  # noqa: F401,E402
from probayes_amd import linreg  # noqa: F401,E402
from probayes_amd.linreg import LinRegConditional  # noqa: F401,E402
