from .fvq import FactorizedVectorQuantize  # noqa: F401
from .rvq import ResidualVQ  # noqa: F401
