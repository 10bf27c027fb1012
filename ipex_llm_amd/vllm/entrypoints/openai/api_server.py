"""``python -m ipex_llm_amd.vllm.entrypoints.openai.api_server --model PATH
--load-in-low-bit sym_int4 [--tensor-parallel-size N]`` (N > 1: under
``torchrun --nproc-per-node N``, one process per GPU; rank 0 serves) -- the
reference's vLLM OpenAI server command
(``SRC/vllm/xpu/entrypoints/openai/api_server.py``) on the native engine:
the model is loaded and converted by ``vllm.engine.IPEXLLMLLMEngine``, the
routes (``/v1/models``, ``/v1/completions``, ``/v1/chat/completions``,
streaming, ``/health``, ``/metrics``) are ``serving.api_server.build_app``'s."""
from __future__ import annotations

import logging

from .cli_args import make_arg_parser, unsupported

log = logging.getLogger("ipex_llm_amd.vllm")


def build_app_from_args(args):
    from ....serving.api_server import build_app
    from ...engine import EngineArgs, IPEXLLMLLMEngine
    ea = EngineArgs(model=args.model, tokenizer=args.tokenizer, dtype=args.dtype,
                    tensor_parallel_size=args.tensor_parallel_size, max_model_len=args.max_model_len,
                    max_num_seqs=args.max_num_seqs, block_size=args.block_size,
                    gpu_memory_utilization=args.gpu_memory_utilization, enforce_eager=args.enforce_eager,
                    enable_prefix_caching=args.enable_prefix_caching, seed=args.seed, device=args.device,
                    trust_remote_code=args.trust_remote_code)
    eng = IPEXLLMLLMEngine.from_engine_args(ea, load_in_low_bit=args.load_in_low_bit)
    name = args.served_model_name or str(args.model)
    app = build_app(eng.engine, eng.tokenizer, name)         # (its lifespan runs the engine loop)
    if args.api_key:
        from starlette.middleware.base import BaseHTTPMiddleware
        from starlette.responses import JSONResponse

        async def check_key(request, call_next):
            if request.url.path.startswith("/v1") and \
                    request.headers.get("Authorization", "") != f"Bearer {args.api_key}":
                return JSONResponse({"error": "Unauthorized"}, status_code=401)
            return await call_next(request)
        app.add_middleware(BaseHTTPMiddleware, dispatch=check_key)
    return app, eng


def main(argv=None):
    args = make_arg_parser().parse_args(argv)
    ign = unsupported(args)
    if ign:
        log.warning("vLLM flags accepted without effect here: %s", ", ".join(ign))
    app, eng = build_app_from_args(args)
    if not eng.is_driver:
        # --tensor-parallel-size N under torchrun: ranks > 0 only execute the
        # driver's (rank 0's) step plans; rank 0 alone serves HTTP
        eng.run_worker()
        return
    import uvicorn
    try:
        uvicorn.run(app, host=args.host, port=args.port)
    finally:
        eng.shutdown()


if __name__ == "__main__":
    main()
