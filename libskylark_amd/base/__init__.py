"""Base layer: context, random streams, distributions, QMC, exceptions, linear algebra."""
from . import distributions, exceptions, quasirand  # noqa: F401
from .context import Context, RandomSamplesArray  # noqa: F401
from .exceptions import *  # noqa: F401,F403
