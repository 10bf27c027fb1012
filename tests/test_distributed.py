"""Multi-process CPU tests (gloo, world_size 2) of the distributed paths:
AutoTP sharding + row-parallel all-reduce, pipeline-parallel generate, and
the collective helpers.  Reference strategy: the reference only exercises
these through example scripts; here they are unit tests."""
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


def _tiny_llama(path, layers=4):
    from transformers import LlamaConfig, LlamaForCausalLM
    torch.manual_seed(0)
    cfg = LlamaConfig(vocab_size=320, hidden_size=128, intermediate_size=256, num_hidden_layers=layers,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=512)
    m = LlamaForCausalLM(cfg).eval()
    m.save_pretrained(path)
    return m


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    from ipex_llm_amd.parallel.comm import init_distributed
    init_distributed("gloo")


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


def _tp_worker(rank, world, port, path, qtype):
    _init(rank, world, port)
    import torch.distributed as dist
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    from transformers import LlamaForCausalLM
    ref = LlamaForCausalLM.from_pretrained(path, torch_dtype=torch.float32).eval()
    ids = torch.randint(0, 320, (2, 9), generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        want = ref(ids).logits.float()
    m = AutoModelForCausalLM.from_pretrained(path, load_in_low_bit=qtype, torch_dtype=torch.float32,
                                             tensor_parallel=True)
    assert m._tp["world"] == world and m._tp["num_heads"] == 4 // world
    # each rank holds 1/world of q rows
    assert m.model.layers[0].self_attn.qkv_proj.out_features == (4 // world + 2 // world) * 32 + 2 // world * 32
    with torch.no_grad():
        got = m(ids).logits.float()
    rel = ((got - want).norm() / want.norm()).item()
    tol = 2e-2 if qtype == "bf16" else 0.3
    assert rel < tol, rel
    g = m.generate(ids, max_new_tokens=4)
    gl = [None] * world
    dist.all_gather_object(gl, g.tolist())
    assert gl[0] == gl[1]                       # ranks agree on every token
    dist.destroy_process_group()


@pytest.mark.parametrize("qtype", ["bf16", "sym_int8"])
def test_tensor_parallel_matches_single(tmp_path, qtype):
    p = str(tmp_path / "m")
    _tiny_llama(p)
    _run(_tp_worker, 2, p, qtype)


def _pp_worker(rank, world, port, path, want):
    _init(rank, world, port)
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    m = AutoModelForCausalLM.from_pretrained(path, load_in_low_bit="sym_int8", torch_dtype=torch.float32,
                                             pipeline_parallel_stages=world)
    assert m._pp["start"] == 2 * rank
    ids = torch.tensor(want["ids"])
    out = m.generate(ids, max_new_tokens=5)
    assert out.tolist() == want["out"], (out.tolist(), want["out"])
    import torch.distributed as dist
    dist.destroy_process_group()


def test_pipeline_parallel_generate_matches_single(tmp_path):
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    p = str(tmp_path / "m")
    _tiny_llama(p)
    ids = torch.randint(0, 320, (2, 7), generator=torch.Generator().manual_seed(3))
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="sym_int8", torch_dtype=torch.float32)
    out = m.generate(ids, max_new_tokens=5, do_sample=False)
    _run(_pp_worker, 2, p, {"ids": ids.tolist(), "out": out.tolist()})


PP_PROMPTS = [list(range(3, 30)), [5, 9, 11], list(range(40, 47)), list(range(100, 161)), [7, 7, 8, 9]]


def _ppw_run(m, world_rank0: bool = True):
    from ipex_llm_amd.serving.engine import SamplingParams
    from ipex_llm_amd.serving.pp_worker import PPModelWorker
    # 2 sequences per slot, one prefill per tick, 16-token prefill chunks:
    # exercises admission, partial prefill and decode in flight together
    w = PPModelWorker(m, max_num_seqs=2, max_prefilled_seqs=1, prefill_chunk=16, max_model_len=128)
    if w.is_head:
        out = w.generate(PP_PROMPTS, SamplingParams(max_new_tokens=6))
        w.stop()
        return out, w.stats
    w.serve_forever()
    return None, w.stats


def _ppw_worker(rank, world, port, path, want):
    _init(rank, world, port)
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    m = AutoModelForCausalLM.from_pretrained(path, load_in_low_bit="sym_int8", torch_dtype=torch.float32,
                                             pipeline_parallel_stages=world)
    out, stats = _ppw_run(m)
    if rank == 0:
        assert out == want, (out, want)
        assert stats["ticks"] > stats["bubbles"]
    import torch.distributed as dist
    dist.destroy_process_group()


def test_pp_serving_worker_matches_single(tmp_path):
    """PPModelWorker (micro-batched pipeline serving, reference
    pipeline_parallel.py:448-927): world 1 and a 2-stage gloo pipeline both
    reproduce the static engine's greedy tokens."""
    from ipex_llm_amd.engine.runner import Engine
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    from ipex_llm_amd.transformers.hf_native import get_native
    p = str(tmp_path / "m")
    _tiny_llama(p)
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="sym_int8", torch_dtype=torch.float32)
    nm, _ = get_native(m)
    ref = Engine(nm).generate(PP_PROMPTS, max_new_tokens=6, use_graph=False)
    want = [r[len(q):] for r, q in zip(ref, PP_PROMPTS)]
    single, _ = _ppw_run(nm)
    assert single == want
    _run(_ppw_worker, 2, p, want)


def _coll_worker(rank, world, port):
    _init(rank, world, port)
    from ipex_llm_amd.parallel import comm
    t = torch.full((4, 8), float(rank + 1))
    r = comm.all_reduce_inplace(t)
    assert torch.all(r == sum(range(1, world + 1)))
    g = comm.all_gather_last_dim(torch.full((2, 3), float(rank)))
    assert g.shape == (2, 3 * world) and g[0, -1].item() == world - 1
    b = comm.broadcast_tensor(torch.tensor([rank * 10]), src=1)
    assert b.item() == 10
    import torch.distributed as dist
    dist.destroy_process_group()


def test_collectives_gloo():
    _run(_coll_worker, 2)


def _ep_worker(rank, world, port, path, want):
    _init(rank, world, port)
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    m = AutoModelForCausalLM.from_pretrained(path, load_in_low_bit="sym_int8", torch_dtype=torch.float32,
                                             expert_parallel=True)
    blk = m.model.layers[0].mlp
    assert blk.experts.num_experts == 4 // world and blk._ep["e0"] == rank * (4 // world)
    ids = torch.tensor(want["ids"])
    with torch.no_grad():
        got = m(ids).logits.float()
    ref = torch.tensor(want["logits"])
    assert ((got - ref).norm() / ref.norm()).item() < 1e-4
    # token-sharded prefill: all-to-all dispatch == replicated compute
    from ipex_llm_amd.parallel.ep import ExactSplitAllToAll, ep_moe_all_to_all
    from ipex_llm_amd.transformers.hf_native import get_native
    nm, _ = get_native(m)
    moe = nm.layers[0].mlp
    x = torch.randn(6, 128, generator=torch.Generator().manual_seed(rank))
    moe.ep_a2a = ExactSplitAllToAll(None, moe.local_experts)
    mine = ep_moe_all_to_all(x, moe)
    assert moe.ep_a2a.last_sent_rows == 6 * 2       # exactly T * k rows leave the rank
    moe.ep_a2a = None
    import torch.distributed as dist
    xs = [torch.empty_like(x) for _ in range(world)]
    dist.all_gather(xs, x)                       # replicated-token reference
    xa = torch.cat(xs)
    w, ids_ = moe.route(xa)
    part = moe._experts_loop(xa, w, ids_)
    dist.all_reduce(part)
    want = part[rank * 6:(rank + 1) * 6]
    assert torch.allclose(mine, want, atol=1e-4), (mine - want).abs().max()
    dist.destroy_process_group()


def test_expert_parallel_matches_single(tmp_path):
    from transformers import Qwen2MoeConfig, Qwen2MoeForCausalLM
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    torch.manual_seed(0)
    cfg = Qwen2MoeConfig(vocab_size=256, hidden_size=128, intermediate_size=128, moe_intermediate_size=64,
                         shared_expert_intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
                         num_key_value_heads=2, num_experts=4, num_experts_per_tok=2, max_position_embeddings=256)
    hf = Qwen2MoeForCausalLM(cfg).eval()
    with torch.no_grad():
        for n, p in hf.named_parameters():
            if p.dim() == 3 or "gate" in n:
                p.normal_(0, 0.05)
    p = str(tmp_path / "moe")
    hf.save_pretrained(p)
    ids = torch.randint(0, 256, (2, 6), generator=torch.Generator().manual_seed(5))
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="sym_int8", torch_dtype=torch.float32)
    with torch.no_grad():
        logits = m(ids).logits.float()
    _run(_ep_worker, 2, p, {"ids": ids.tolist(), "logits": logits.tolist()})


def _ppw_fail_worker(rank, world, port, path):
    _init(rank, world, port)
    import time
    from ipex_llm_amd.parallel.health import RankFailureError
    from ipex_llm_amd.serving.engine import SamplingParams
    from ipex_llm_amd.serving.pp_worker import PPModelWorker
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    m = AutoModelForCausalLM.from_pretrained(path, load_in_low_bit="sym_int8", torch_dtype=torch.float32,
                                             pipeline_parallel_stages=world)
    w = PPModelWorker(m, max_num_seqs=2, max_model_len=128).enable_failure_detection(timeout=3.0, interval=0.2)
    if rank == 1:
        n = [0]
        orig = w._tick

        def dying_tick(ctrl):
            n[0] += 1
            if n[0] == 4:
                os._exit(0)                      # the stage process vanishes mid-generation
            return orig(ctrl)
        w._tick = dying_tick
        w.serve_forever()
        os._exit(0)
    t0 = time.time()
    try:
        w.generate([list(range(3, 20)), [5, 6, 7]], SamplingParams(max_new_tokens=60))
        raise AssertionError("generation finished although stage 1 died")
    except RankFailureError as e:
        assert "rank" in str(e) or "collective" in str(e), e
    assert time.time() - t0 < 60
    assert all(sq.done and sq.finish_reason.startswith("error") for sq in w.seqs.values())
    assert w.health()["status"] == "error"
    os._exit(0)                                  # (no teardown collective with a dead peer)


def test_pp_serving_detects_dead_rank(tmp_path):
    """§5.3 failure detection: a pipeline stage dying mid-generation fails the
    in-flight requests with an error on rank 0 (heartbeats + collective
    error), instead of blocking until the process-group timeout"""
    p = str(tmp_path / "m")
    _tiny_llama(p)
    _run(_ppw_fail_worker, 2, p)


def test_rank_monitor_heartbeats(tmp_path):
    import time
    import torch.distributed as dist
    from ipex_llm_amd.parallel.health import Heartbeat, RankFailureError, RankMonitor
    store = dist.FileStore(str(tmp_path / "store"), 1)
    hb = Heartbeat(store, 1, interval=0.05).start()
    mon = RankMonitor(store, [1, 2], timeout=0.5, poll=0.0)
    time.sleep(0.6)
    assert mon.poll_now() == [2]                 # rank 2 never beat
    mon.ranks = [1]
    mon.check()                                  # rank 1 alive
    hb._stop.set()                               # rank 1 freezes (no clean stop)
    time.sleep(0.7)
    try:
        mon.check()
        raise AssertionError("stale heartbeat not detected")
    except RankFailureError as e:
        assert "[1]" in str(e)
    hb2 = Heartbeat(store, 3, interval=0.05).start()
    hb2.stop()                                   # clean stop is not a failure
    assert RankMonitor(store, [3], timeout=0.1, poll=0.0).poll_now() == []


def _tp_save_worker(rank, world, port, path, out_dir):
    _init(rank, world, port)
    import torch.distributed as dist
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    ids = torch.randint(0, 320, (1, 9), generator=torch.Generator().manual_seed(1))
    m = AutoModelForCausalLM.from_pretrained(path, load_in_low_bit="sym_int4", torch_dtype=torch.float32,
                                             tensor_parallel=True)
    with torch.no_grad():
        a = m(ids).logits
    m.save_low_bit(out_dir)
    assert os.path.exists(os.path.join(out_dir, f"model-tp{rank:02d}-of-{world:02d}.safetensors"))
    m2 = AutoModelForCausalLM.load_low_bit(out_dir, torch_dtype=torch.float32, tensor_parallel=True)
    assert m2._tp["world"] == world and m2._tp["rank"] == rank
    with torch.no_grad():
        b = m2(ids).logits
    assert torch.allclose(a, b, atol=1e-5), (a - b).abs().max()
    dist.destroy_process_group()


def test_tp_per_rank_save_and_load(tmp_path):
    """§5.4: a tensor-parallel model saves one shard per rank and loads back
    on the same world size without re-sharding the dense checkpoint"""
    p = str(tmp_path / "m")
    _tiny_llama(p)
    _run(_tp_save_worker, 2, p, str(tmp_path / "tp_saved"))
    import json
    meta = json.load(open(tmp_path / "tp_saved" / "illm_low_bit.json"))
    assert meta["tensor_parallel"] == 2
