"""Low-bit formats: qtype registry, quantizers and layout conversion."""
from .qtypes import (ggml_tensor_qtype, gguf_mixed_qtype, get_format, resolve_qtype, qtype_name,  # noqa: F401
                     is_dense, get_block_size, QFormat)
