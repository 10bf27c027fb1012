"""Device / host capability probes (reference ``transformers/utils.py:141-183``
get_xpu_device_name -> arc/pvc/mtl..., ``utils/isa_checker.py``)."""
from __future__ import annotations

import functools
import platform


@functools.lru_cache(None)
def gpu_arch(device: int = 0) -> str:
    """'gfx950' on MI355X; '' without a GPU."""
    import torch
    if not torch.cuda.is_available():
        return ""
    props = torch.cuda.get_device_properties(device)
    return getattr(props, "gcnArchName", "").split(":")[0]


def get_device_name(device: int = 0) -> str:
    """Coarse device class used by heuristics (reference returns arc/pvc/...)."""
    a = gpu_arch(device)
    if a.startswith("gfx95"):
        return "mi355x"
    if a.startswith("gfx94"):
        return "mi300"
    return "cpu" if not a else a


@functools.lru_cache(None)
def cpu_flags() -> frozenset:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("flags"):
                    return frozenset(line.split(":", 1)[1].split())
    except OSError:
        pass
    return frozenset()


def check_avx2() -> bool:
    return "avx2" in cpu_flags()


def check_avx512() -> bool:
    return "avx512f" in cpu_flags()


def is_server() -> bool:
    return check_avx512()
