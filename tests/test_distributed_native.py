"""Native decoder under tensor / expert parallelism (gloo, CPU, world 2/4/8).

``random_native_model(..., tp_group=...)`` / ``ep_group=`` shard one set of
random weights (same seed on every rank) exactly like bench.py --tp / --ep,
and the native decode engine must reproduce the single-process model's greedy
tokens.  The reference validates AutoTP only with example scripts on real
multi-GPU machines; here every rank count up to a full 8-GPU node
is rehearsed on CPU processes.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(fn, world, *args):
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=fn, args=(r, world, port) + args) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert codes == [0] * world, f"worker exit codes {codes}"


def _llama_cfg():
    from transformers import LlamaConfig
    return LlamaConfig(vocab_size=256, hidden_size=512, intermediate_size=1024, num_hidden_layers=2,
                       num_attention_heads=8, num_key_value_heads=2, max_position_embeddings=512)


def _mixtral_cfg():
    from transformers import MixtralConfig
    return MixtralConfig(vocab_size=256, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                         num_attention_heads=4, num_key_value_heads=2, num_local_experts=8, num_experts_per_tok=2,
                         max_position_embeddings=512)


PROMPTS = [[3, 14, 15, 92, 65, 35], [27, 18, 28, 18, 28, 45, 90, 45]]


def _generate(model):
    from ipex_llm_amd.engine.runner import Engine
    return Engine(model).generate(PROMPTS, max_new_tokens=6, use_graph=False)


def _worker(rank, world, port, kind, want):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    import torch.distributed as dist
    from ipex_llm_amd.parallel.comm import init_distributed
    init_distributed("gloo")
    from ipex_llm_amd.models.builder import random_native_model
    g = dist.group.WORLD
    if kind == "tp":
        m = random_native_model(_llama_cfg(), "sym_int8", "cpu", torch.float32, seed=0, std=0.05, tp_group=g)
        assert m.spec.num_heads == 8 // world and m.tp_group is g
        assert m.layers[0].self_attn.o_proj.mp_group is g and m.layers[0].mlp.down_proj.mp_group is g
    elif kind == "ep":
        m = random_native_model(_mixtral_cfg(), "sym_int8", "cpu", torch.float32, seed=0, std=0.05, ep_group=g)
        moe = m.layers[0].mlp
        assert moe.local_experts == 8 // world and moe.e0 == rank * (8 // world)
    else:
        # token-sharded EP: rank r serves ONLY prompt r % 2 (attention is not
        # replicated); its MoE pairs travel through the exact-split exchange
        from ipex_llm_amd.parallel.ep import ExactSplitAllToAll
        m = random_native_model(_mixtral_cfg(), "sym_int8", "cpu", torch.float32, seed=0, std=0.05, ep_group=g,
                                ep_tokens=True)
        a2a = m.layers[0].mlp.ep_a2a
        assert isinstance(a2a, ExactSplitAllToAll) and m.layers[1].mlp.ep_a2a is a2a
        from ipex_llm_amd.engine.runner import Engine
        out = Engine(m).generate([PROMPTS[rank % 2]], max_new_tokens=6, use_graph=False)
        assert a2a.last_sent_rows == 1 * 2          # last call: one decode token x top-2, nothing more
        assert out == [want[rank % 2]], (rank, out, want)
        dist.destroy_process_group()
        return
    out = _generate(m)
    assert out == want, (rank, out, want)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_native_tp_decode_matches_single(world):
    from ipex_llm_amd.models.builder import random_native_model
    single = random_native_model(_llama_cfg(), "sym_int8", "cpu", torch.float32, seed=0, std=0.05)
    _run(_worker, world, "tp", _generate(single))


@pytest.mark.parametrize("world", [2, 4])
def test_native_ep_decode_matches_single(world):
    from ipex_llm_amd.models.builder import random_native_model
    single = random_native_model(_mixtral_cfg(), "sym_int8", "cpu", torch.float32, seed=0, std=0.05)
    _run(_worker, world, "ep", _generate(single))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_native_ep_token_sharded_matches_single(world):
    from ipex_llm_amd.models.builder import random_native_model
    single = random_native_model(_mixtral_cfg(), "sym_int8", "cpu", torch.float32, seed=0, std=0.05)
    _run(_worker, world, "ep_a2a", _generate(single))


def _serve_tp_worker(rank, world, port, want):
    """tensor-parallel serving (LLMEngine over a TP-sharded native model):
    rank 0 runs the scheduler with two concurrent requests and broadcasts each
    step's plan; the other ranks replay it in run_worker()"""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    import torch.distributed as dist
    from ipex_llm_amd.parallel.comm import init_distributed
    init_distributed("gloo")
    from ipex_llm_amd.models.builder import random_native_model
    from ipex_llm_amd.serving.engine import LLMEngine, SamplingParams
    g = dist.group.WORLD
    m = random_native_model(_llama_cfg(), "sym_int8", "cpu", torch.float32, seed=0, std=0.05, tp_group=g)
    eng = LLMEngine(m, max_batch=4, max_model_len=128, block_size=64)
    assert eng.tp_world == world and eng.is_driver == (rank == 0)
    if rank == 0:
        sp = SamplingParams(max_new_tokens=6)
        rids = [eng.add_request(p, sp) for p in PROMPTS]      # two concurrent requests
        while any(not eng.requests[r].finished for r in rids):
            eng.step()
        out = [eng.requests[r].generated for r in rids]
        eng.shutdown()
        assert out == want, (out, want)
    else:
        eng.run_worker()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_tp_serving_engine_matches_single(world):
    """vLLM --tensor-parallel-size equivalent on the serving engine: the TP
    group's greedy tokens == the unsharded serving engine's"""
    from ipex_llm_amd.models.builder import random_native_model
    from ipex_llm_amd.serving.engine import LLMEngine, SamplingParams
    single = random_native_model(_llama_cfg(), "sym_int8", "cpu", torch.float32, seed=0, std=0.05)
    want = LLMEngine(single, max_batch=4, max_model_len=128, block_size=64).generate(
        PROMPTS, SamplingParams(max_new_tokens=6))
    _run(_serve_tp_worker, world, want)


def test_tp_plan_encoding_round_trip():
    from ipex_llm_amd.serving.engine import LLMEngine
    pre = [([5, 6, 7, 8, 9], 2, [3, 4]), ([1, 2], 0, [7])]
    dec = [(11, 40, [0, 1, 2]), (12, 3, [9])]
    words = LLMEngine.encode_plan(pre, dec)
    p2, d2 = LLMEngine.decode_plan(words)
    assert [(t[s:], s, b) for t, s, b in p2] == [(t[s:], s, b) for t, s, b in pre]
    assert [len(t) for t, _, _ in p2] == [5, 2]
    assert d2 == dec and LLMEngine.decode_plan([0]) is None
