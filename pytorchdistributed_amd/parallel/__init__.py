"""Parallelism wrappers."""
from .ddp import DistributedDataParallel, DDP  # noqa: F401
from .flat import FlatGroup  # noqa: F401
from .param_server import ParameterServer  # noqa: F401
