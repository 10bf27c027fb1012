"""Measured GEMM dispatch bookkeeping (ops/gemm.py _pick): row buckets and the
cached per-shape choice (the timing itself needs a GPU: tests/test_gpu_kernels.py)."""
from ipex_llm_amd.ops import gemm as G


def test_row_buckets():
    assert [G._mbucket(m) for m in (1, 512, 513, 1024, 1025, 8192)] == [1, 512, 1024, 1024, 2048, 8192]


def test_cached_choice_is_shared_within_a_bucket():
    saved = dict(G._CHOICE)
    try:
        G._CHOICE.clear()
        G._CHOICE[(1024, 4096, 4096, False, 0)] = "lib"
        never = lambda: (_ for _ in ()).throw(AssertionError("timed a cached shape"))  # noqa: E731
        assert G._pick((700, 4096, 4096, False, 0), never, never) == "lib"
        assert G._pick((1024, 4096, 4096, False, 0), never, never) == "lib"
        assert G.gemm_choices() == {(1024, 4096, 4096, False, 0): "lib"}
    finally:
        G._CHOICE.clear()
        G._CHOICE.update(saved)
