"""Error helpers, lazy imports, logging (reference ``SRC/utils/common/*``:
invalidInputError / invalidOperationError, LazyImport, MuteHFLogger)."""
from __future__ import annotations

import contextlib
import importlib
import logging

logger = logging.getLogger("ipex_llm_amd")


def invalidInputError(condition: bool, err: str, fix: str = ""):
    if not condition:
        msg = err + (f" -- {fix}" if fix else "")
        logger.error(msg)
        raise ValueError(msg)


def invalidOperationError(condition: bool, err: str, fix: str = "", cause: Exception = None):
    if not condition:
        msg = err + (f" -- {fix}" if fix else "")
        logger.error(msg)
        raise RuntimeError(msg) from cause


class LazyImport:
    """Import a module on first attribute access."""

    def __init__(self, name: str):
        self._name, self._mod = name, None

    def __getattr__(self, item):
        if self._mod is None:
            self._mod = importlib.import_module(self._name)
        return getattr(self._mod, item)


@contextlib.contextmanager
def MuteHFLogger(logger_name: str = "transformers", level=logging.ERROR):
    lg = logging.getLogger(logger_name)
    old = lg.level
    lg.setLevel(level)
    try:
        yield
    finally:
        lg.setLevel(old)
