"""Utilities: settings, error helpers, device probes, benchmark wrapper."""
from .common import LazyImport, MuteHFLogger, invalidInputError, invalidOperationError  # noqa: F401
from .settings import Settings, get_settings  # noqa: F401
from .benchmark import BenchmarkWrapper  # noqa: F401
