"""Expert-parallel peer all-to-all (csrc/hip/ep_a2a.hip, parallel/ep.py
EPAllToAll) on the GPU.

The 1-GPU test box cannot run an 8-GPU job, so 2 processes share cuda:0:
they exchange hipIpc handles over a gloo group exactly as ranks on separate
GPUs do (ILLM_EP_P2P=force) and run the same kernels (peer stores then land
in local HBM instead of going over xGMI).  Covered:
  * the exchange itself against a torch reference (expert fn = per-expert
    scaling), exact row count per rank (T*k), counts per source, repeated
    calls with changing T (region reuse / epochs), hipGraph capture + replay;
  * a token-sharded Mixtral-shaped model (each rank its OWN prompt) against
    the single-process model of the same seed: prefill logits, and captured
    decode == eager decode;
  * a missing peer: ERR_PEER in the kernel error word and NaN output instead
    of a hang or stale rows.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _mixtral_cfg():
    from transformers import MixtralConfig
    return MixtralConfig(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                         num_attention_heads=4, num_key_value_heads=2, num_local_experts=4, num_experts_per_tok=2,
                         max_position_embeddings=512, rms_norm_eps=1e-5)


def _exchange(rank, world):
    from ipex_llm_amd.parallel.ep import EPAllToAll
    H, k, E = 256, 2, 4 * world
    el = E // world
    a2a = EPAllToAll(None, H, max_tokens=64, top_k=k, experts_per_rank=el, dtype=torch.bfloat16, device="cuda:0")

    def expert_fn(rx, re):                     # expert e scales its rows by (e + 1)
        return (rx.float() * (re.float() + 1).clamp(min=0)[:, None]).to(rx.dtype)

    for it, T in enumerate((5, 64, 1, 33)):
        g = torch.Generator(device="cuda").manual_seed(100 * it + rank)
        x = torch.randn(T, H, generator=g, device="cuda").to(torch.bfloat16)
        ids = torch.stack([torch.randperm(E, generator=g, device="cuda")[:k] for _ in range(T)]).to(torch.int32)
        w = torch.rand(T, k, generator=g, device="cuda")
        y = a2a(x, w, ids, expert_fn)
        want = (x.float()[:, None, :] * (ids.float() + 1)[:, :, None] * w[:, :, None]).sum(1)
        err = ((y.float() - want).abs().max() / want.abs().max()).item()
        assert err < 2e-2, (it, T, err)
        assert a2a.last_sent_rows == T * k, (a2a.last_sent_rows, T * k)
    # graph capture: epochs and counts are device-resident
    T = 16
    x = torch.randn(T, H, device="cuda").to(torch.bfloat16)
    ids = ((torch.arange(T * k, device="cuda") + rank) % E).view(T, k).to(torch.int32)
    w = torch.full((T, k), 0.5, device="cuda")
    a2a(x, w, ids, expert_fn)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        y = a2a(x, w, ids, expert_fn)
    for v in range(3):
        x.copy_(torch.randn(T, H, device="cuda").to(torch.bfloat16))
        graph.replay()
        torch.cuda.synchronize()
        want = (x.float()[:, None, :] * (ids.float() + 1)[:, :, None] * 0.5).sum(1)
        assert ((y.float() - want).abs().max() / want.abs().max()).item() < 2e-2, v
    import ipex_llm_amd.ops as ops
    ops.check_kernel_errors()
    return a2a


def _model(rank, world):
    from ipex_llm_amd.engine.runner import Engine
    from ipex_llm_amd.models.builder import random_native_model
    from ipex_llm_amd.models.cache import SequenceState
    import torch.distributed as dist
    cfg = _mixtral_cfg()
    single = random_native_model(cfg, "sym_int4", "cuda:0", torch.bfloat16, seed=3)
    m = random_native_model(cfg, "sym_int4", "cuda:0", torch.bfloat16, seed=3, ep_group=dist.group.WORLD,
                            ep_tokens=True, ep_max_tokens=256)
    a2a = m.layers[0].mlp.ep_a2a
    assert a2a is not None and a2a.capturable and type(a2a).__name__ == "TieredAllToAll"   # decode + prefill tiers
    g = torch.Generator().manual_seed(11 + rank)                 # every rank its own prompts
    prompts = torch.randint(0, cfg.vocab_size, (2, 48), generator=g)
    logits = {}
    for name, mod in (("single", single), ("ep", m)):
        eng = Engine(mod)
        eng._ensure_cache(2, 128)
        seqs = [SequenceState(eng.cache.allocator.alloc(2)) for _ in range(2)]
        logits[name] = eng.prefill_batch(seqs, prompts.cuda()).float()
        if name == "ep":                         # captured decode == eager decode through the exchange
            cur = torch.argmax(logits[name], -1)
            lens = torch.tensor([s.length for s in seqs], device="cuda")
            outs = {}
            for use_graph in (False, True):
                for s in seqs:
                    s.length = 48
                st = eng.decode_step_obj(seqs, 128, greedy=True, use_graph=use_graph)
                st.set_state(cur.clone(), lens.clone())
                toks = []
                for _ in range(4):
                    st.step()
                    toks.append(st.next_ids.clone())
                outs[use_graph] = torch.stack(toks).tolist()
            assert outs[True] == outs[False], outs
    a, b = logits["ep"], logits["single"]
    rel = ((a - b).norm() / b.norm()).item()
    assert rel < 3e-2, rel
    import ipex_llm_amd.ops as ops
    ops.check_kernel_errors()


def _worker(rank, world, port, q, what):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ILLM_EP_P2P="force",
                          ILLM_EP_TIMEOUT_S="2")
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        if what == "exchange":
            _exchange(rank, world).close()
        elif what == "model":
            _model(rank, world)
        else:                                    # rank 1 never calls: rank 0 must fail loudly
            from ipex_llm_amd.parallel.ep import EPAllToAll
            import ipex_llm_amd.ops as ops
            a2a = EPAllToAll(None, 64, max_tokens=8, top_k=1, experts_per_rank=1, dtype=torch.bfloat16,
                             device="cuda:0")
            if rank == 0:
                x = torch.ones(4, 64, device="cuda", dtype=torch.bfloat16)
                ids = torch.tensor([[0], [1], [1], [0]], dtype=torch.int32, device="cuda")
                y = a2a(x, torch.ones(4, 1, device="cuda"), ids, lambda rx, re: rx)
                torch.cuda.synchronize()
                assert torch.isnan(y[1].float()).all(), y
                try:
                    ops.check_kernel_errors()
                    raise AssertionError("missing peer not reported")
                except ops.KernelError as e:
                    assert "peer" in str(e), e
            dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))
        raise


@pytest.mark.parametrize("what", ["exchange", "model", "missing_peer"])
def test_ep_all_to_all_procs_one_gpu(what):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, what)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(150)
    res = dict(q.get(timeout=5) for _ in range(world))
    for p in ps:
        if p.is_alive():
            p.kill()
    assert all(v == "ok" for v in res.values()), res
