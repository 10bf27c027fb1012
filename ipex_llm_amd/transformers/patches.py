"""Remote-code import filter (reference ``SRC/transformers/patches.py:23``):
remote modelling files that import ``flash_attn`` (a CUDA-only package) are
still loadable -- the import is dropped from the dependency check, and their
attention falls back to eager / SDPA paths."""
from __future__ import annotations

import contextlib
from typing import List

_DROP = ("flash_attn",)


def patch_flash_attn_import(filename: str) -> List[str]:
    from transformers.dynamic_module_utils import get_imports
    return [i for i in get_imports(filename) if i not in _DROP]


@contextlib.contextmanager
def remote_code_patches():
    """Context manager used around ``from_pretrained(trust_remote_code=True)``."""
    import transformers.dynamic_module_utils as dmu
    orig = dmu.get_imports

    def filtered(filename):
        return [i for i in orig(filename) if i not in _DROP]

    dmu.get_imports = filtered
    try:
        yield
    finally:
        dmu.get_imports = orig
